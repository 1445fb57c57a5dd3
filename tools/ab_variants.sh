#!/bin/bash
# Profile bench.py under the default module and under variant builds
# (tools/build_variant.sh NAME ... ; cp bench.py build/var_NAME/), one
# rocprofv3 kernel trace each, and print the matching kernels' step timeline:
#   OUT=r6x VARIANTS="base wd8" ARGS="--model ref --steps 5 --warmup 2" KPAT="wres|step" bash tools/ab_variants.sh
# (a variant named NAME=FLAGS runs the default module under MCC_AB=FLAGS)
set -o pipefail
R=$PWD; O=$R/gpurun_out/${OUT:-ab}; mkdir -p $O; export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  B=$R/bench.py; E=""
  case $v in base) ;; *=*) E=${v#*=} ;; *) B=$R/build/var_$v/bench.py ;; esac
  d=${v%%=*}
  (cd /tmp && MCC_AB=$E timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$d -o run --output-format csv -- \
     python3 $B ${ARGS:---steps 5 --warmup 2} --eager-anchor off --no-dist > $O/$d.log 2>&1) || { echo "$v failed"; tail $O/$d.log; exit 1; }
  echo "== $v"; python3 $R/tools/step_timeline.py $O/$d/run_kernel_trace.csv | grep -E "${KPAT:-.}"
done
