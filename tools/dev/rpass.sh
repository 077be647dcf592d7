#!/bin/bash
# Dev: per-kernel VGPR / AGPR / scratch / occupancy of one csrc/*.hip file (hipcc resource-usage remarks)
# usage: tools/dev/rpass.sh conv_gemm [grep-pattern]
f=$1; pat=${2:-.}
hipcc -O3 -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I"$(dirname "$0")/../../csrc" -c "$(dirname "$0")/../../csrc/$f.hip" \
  -o /tmp/rpass_$f.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import re, sys
cur = None
rows = []
for l in sys.stdin:
    m = re.search(r'Function Name: (\S+)', l)
    if m:
        cur = {'name': m.group(1)}; rows.append(cur); continue
    m = re.search(r'remark:\s+([A-Za-z \[\]/]+): (\d+)', l)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
for r in rows:
    if re.search(sys.argv[1], r['name']):
        print(r['name'][:90], 'VGPR', r.get('VGPRs'), 'AGPR', r.get('AGPRs'), 'spill', r.get('VGPRs Spill'),
              'scratch', r.get('ScratchSize [bytes/lane]'), 'occ', r.get('Occupancy [waves/SIMD]'), 'LDS', r.get('LDS Size [bytes/block]'))
" "$pat"
