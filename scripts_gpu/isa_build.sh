#!/bin/bash
# hipcc --save-temps of one csrc file (build.py flags) into /tmp/isa/<tag>/, then the
# resource usage and the static ISA census (isa_stats.py) of the kernels matching $3.
# Usage: isa_build.sh FILE.hip TAG KERNEL_SUBSTRING
P=/root/repo/140-extdm-distribution-extrapolation-diffusion-model-for-video-prediction_amd
F=$1; TAG=$2; K=$3
mkdir -p /tmp/isa/$TAG && cd /tmp/isa/$TAG || exit 1
EXTRA=""
case $F in stw_x3.hip|stw64_x3.hip|cross_x3.hip) EXTRA="-fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1";; attn_core.hip) EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1";; xpath_x3.hip) EXTRA="-fno-slp-vectorize";; esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I /root/repo/include -I $P/csrc $EXTRA \
  --save-temps -Rpass-analysis=kernel-resource-usage -c $P/csrc/$F -o out.o 2> remarks.txt || { cat remarks.txt | grep error; exit 1; }
S=$(ls *-hip-amdgcn-amd-amdhsa-gfx950.s)
grep -A8 "Function Name: .*$K" remarks.txt | grep -E "VGPRs:|AGPRs|Scratch|Occupancy" | sed 's/.*remark: *//; s/ \[-Rpass.*//' | tr '\n' ' '; echo
python /root/repo/scripts_gpu/isa_stats.py $S $K
