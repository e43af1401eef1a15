#!/bin/bash
# Summarise per-kernel VGPR / scratch / occupancy / LDS from hipcc's resource remarks.
# usage: tools/resources.sh file.hip [extra hipcc flags]
f=$1; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c "$f" -o /tmp/_res.o -Rpass-analysis=kernel-resource-usage "$@" 2>&1 \
 | awk '/Function Name:/{n=$NF} /VGPRs: [0-9]/{v=$3} /ScratchSize/{s=$NF} /Occupancy/{o=$NF} /LDS Size/{l=$NF; printf "%-90s vgpr=%s scratch=%s occ=%s lds=%s\n", n, v, s, o, l} /error/{print}' \
 | sed 's/\[-Rpass-analysis=kernel-resource-usage\]//g'
