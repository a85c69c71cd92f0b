#!/bin/bash
set -o pipefail
OUT=gpurun_out/place_prof
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c2 -o c2 --output-format csv -- python tools/place_prof.py > $OUT/c2.log 2>&1 || { tail $OUT/c2.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o c3 --output-format csv -- python tools/place_prof.py c3 > $OUT/c3.log 2>&1 || { tail $OUT/c3.log; exit 2; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/c5 -o c5 --output-format csv -- python tools/place_prof.py c5 > $OUT/c5.log 2>&1 || { tail $OUT/c5.log; exit 3; }
grep placement $OUT/c2.log $OUT/c3.log $OUT/c5.log
for f in $(find $OUT -name "*kernel_stats.csv"); do echo $f; head -8 $f | cut -c1-200; done
