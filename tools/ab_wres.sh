set -o pipefail
R=$PWD; O=$R/gpurun_out/r6z; mkdir -p $O; export TMPDIR=/tmp
for v in base cfg2; do
  B=$R/bench.py; [ $v = base ] || B=$R/build/var_$v/bench.py
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $B --model ref --steps 5 --warmup 2 --eager-anchor off --no-dist > $O/$v.log 2>&1) || { echo "$v failed"; tail $O/$v.log; exit 1; }
  echo "== $v"; python3 $R/tools/step_timeline.py $O/$v/run_kernel_trace.csv | grep -E "wres|step"
done
