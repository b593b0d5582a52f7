#!/bin/bash
# The phase conv's bank-conflict-free lane order (_variants/lrot) against the shipped library: BAIR
# eps bitwise equal across the two, the phase parity tests on the variant, layer 0 interleaved, the
# SQ pass of layer 0 on the variant, whole BAIR DDIM-20 steps interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
VL=$PWD/_variants/${VAR:-lrot}/libextdm_hip.so
timeout -k 10 120 python scripts_gpu/eps_dump.py gpurun_out/eps_A.pt || exit 1
EXTDM_LIB=$VL timeout -k 10 120 python scripts_gpu/eps_dump.py gpurun_out/eps_B.pt || exit 1
python -c "import torch; a=torch.load('gpurun_out/eps_A.pt'); b=torch.load('gpurun_out/eps_B.pt'); print('eps bitwise equal:', torch.equal(a, b), (a-b).abs().max().item())"
EXTDM_LIB=$VL timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fea_phase or unet_forward_vs_reference_golden" -x -q --timeout 300 --timeout-method thread > gpurun_out/lrot_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/lrot_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  timeout -k 10 120 python -u scripts_gpu/layers.py 128 20 f16x3 0 2>&1 | grep layer | sed "s/^/A$rep /" || exit 1
  EXTDM_LIB=$VL timeout -k 10 120 python -u scripts_gpu/layers.py 128 20 f16x3 0 2>&1 | grep layer | sed "s/^/B$rep /" || exit 1
done
for rep in 1 2; do
  for arm in A B; do
    if [ $arm = A ]; then envs="X=0"; else envs="EXTDM_LIB=$VL"; fi
    env $envs timeout -k 10 300 python bench.py --sampling-steps 20 --steps 20 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/lrot_$arm$rep.json 2> gpurun_out/lrot_$arm$rep.err || { tail -5 gpurun_out/lrot_$arm$rep.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/lrot_$arm$rep.json').read().strip().splitlines()[-1]); print('bair', '$arm$rep', d['ms_per_step'], d['value'])"
  done
done
EXTDM_LIB=$VL LAYER=0 TAG=lrotsq bash scripts_gpu/pmc_sq.sh > gpurun_out/lrot_sq_l0.txt 2>&1 || exit 1
