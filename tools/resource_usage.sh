#!/bin/bash
# Per-kernel VGPR / scratch / LDS / occupancy of a csrc file (gfx950): tools/resource_usage.sh csrc/calib.hip
f=$(readlink -f "$1")
d=$(dirname "$f")
(cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -I"$d" -x hip -c "$f" -o /tmp/ru.o -Rpass-analysis=kernel-resource-usage 2>&1) \
 | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|LDS Size|Occupancy" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' \
 | awk '/Function Name/{if(line)print line; line=$3; next}{line=line" | "$0}END{print line}' | c++filt
