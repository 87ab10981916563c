#!/bin/bash
# Per-kernel resource usage (VGPR/AGPR/LDS/occupancy) of a .hip file: scripts/kres.sh csrc/kernels/lenet.hip
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Icsrc -c "$1" -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/{printf "\n%s", substr($3,1,60)} /VGPRs:|AGPRs:|LDS Size|Occupancy|ScratchSize/{printf " | %s", $0}' ; echo
