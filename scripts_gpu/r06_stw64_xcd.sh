#!/bin/bash
# r06: XCD-contiguous workgroup order in stw64_x3 (EXTDM_STW64_XCD=0: dispatch order), layer 6 of
# KTH / Cityscapes / UCF interleaved twice, KTH layer 6 WRITE_SIZE / FETCH_SIZE both ways, the
# window-64 attention tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn.py -x -q --timeout 200 --timeout-method thread -k "window64 or dim16" > gpurun_out/stw64_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/stw64_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for c in kth cityscapes ucf; do
    EXTDM_STW64_XCD=0 timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6 || exit 1
    timeout -k 10 120 python scripts_gpu/layers_cfg.py $c 6 || exit 1
  done
done
for x in 0 1; do
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmcx_$x_$C
    EXTDM_STW64_XCD=$x timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcx_${x}_$C -o run --output-format csv -- python scripts_gpu/pmc_layer_run.py kth 6 10 > gpurun_out/pmcx_${x}_$C.log 2>&1 || exit 1
    f=$(find gpurun_out/pmcx_${x}_$C -name "*counter_collection.csv" | head -1)
    python - "$f" $C $x <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'stw64' in r.get('Kernel_Name', '')]
vals = [float(r['Counter_Value']) for r in rows]
print(f'XCD={sys.argv[3]} {sys.argv[2]}: {len(vals)} records, mean {sum(vals)/max(1,len(vals)):.4g} per record-dispatch')
PY
    find gpurun_out/pmcx_${x}_$C -name "*trace*.csv" -delete
  done
done
