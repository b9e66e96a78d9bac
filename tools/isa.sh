#!/bin/bash
# Device assembly of kernels_mc.hip with the Makefile's flags -> /tmp/isa/kmc.s,
# then the histogram / class map of one kernel: tools/isa.sh KERNEL_SUBSTR [map]
set -e
cd "$(dirname "$0")/../channel-estimation_amd"
mkdir -p /tmp/isa
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form=1 \
    -I../include -Icsrc --cuda-device-only -S csrc/kernels_mc.hip -o /tmp/isa/kmc.s 2>&1 | grep -v hip-link || true
python3 ../tools/isa_hist.py /tmp/isa/kmc.s "$1" 25 --dump /tmp/isa/k.s
awk "/amdhsa_kernel .*$1/,/end_amdhsa_kernel/" /tmp/isa/kmc.s | grep -E "next_free_vgpr|private_segment_fixed|accum_offset|group_segment" | head -4
[ "$2" = map ] && python3 ../tools/isa_map.py /tmp/isa/k.s
exit 0
