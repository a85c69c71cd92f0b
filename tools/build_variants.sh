#!/bin/bash
# Measurement builds of the engine with k_mat ablation / tuning macros: koordinator_amd/lib/variants/<name>.so
# Usage: tools/build_variants.sh name:"-DFLAG=.. -DFLAG2=.." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p koordinator_amd/lib/variants
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  hipcc -O3 -fPIC -std=c++17 -ffp-contract=off --offload-arch=gfx950 $flags -c koordinator_amd/csrc/kg_engine.hip -o /tmp/kgv_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  hipcc -shared --offload-arch=gfx950 /tmp/kgv_$name.o koordinator_amd/lib/obj/kg_host.o koordinator_amd/lib/obj/kg_cpuset.o -o koordinator_amd/lib/variants/$name.so
done
ls -la koordinator_amd/lib/variants
