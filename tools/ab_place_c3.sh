#!/bin/bash
# Config-3 placement throughput (tools/place_prof.py c3) of the default build and measurement builds in
# koordinator_amd/lib/variants, interleaved twice.  Usage: tools/ab_place_c3.sh <variant>...
set -o pipefail
export TMPDIR=/tmp
for r in 1 2; do
  for v in base "$@"; do
    so=koordinator_amd/lib/variants/$v.so; [[ $v == base ]] && so=koordinator_amd/lib/libkoordgpu.so
    KG_ENGINE_SO=$so timeout -k 10 120 python tools/place_prof.py c3 | sed "s/^/$v /" || exit 2
  done
done
