#!/bin/bash
# Register / spill / scratch summary of the megakernel instantiations (device-only compile of
# pt_kernels.hip to assembly; no GPU needed).  Usage: scripts/isa_stats.sh [extra hipcc flags]
set -e
cd "$(dirname "$0")/../dxrpathtracer_amd/csrc"
OUT=${ISA_OUT:-/tmp/isa}
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -Wno-unused-function --cuda-device-only -S "$@" \
  pt_kernels.hip -o $OUT/pt.s
python3 - "$OUT/pt.s" <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r"- \.agpr_count:.*?\.name:\s+(\S+).*?\.private_segment_fixed_size:\s+(\d+).*?\.vgpr_count:\s+(\d+)\s+\.vgpr_spill_count:\s+(\d+)", s, re.S):
    n = m.group(1)
    if re.search(r"k_path|k_bake|k_shade|k_trace|k_shadow", n):
        print(f"{n[:60]:60s} vgpr {m.group(3):>4s} spill {m.group(4):>4s} scratch {m.group(2):>4s}")
PY
