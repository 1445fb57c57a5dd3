#!/bin/bash
# One GPU-box job, parametrised by environment (run through gpurun):
#   OUT=name           results under gpurun_out/<name>/
#   TESTS="args"       pytest arguments (-m gpu is added); empty: skip
#   BENCH="a;b;..."    bench.py argument sets, one JSON line each (leading NAME=value
#                      words are that run's environment, e.g. "MCC_AB=no_lenet --steps 20")
#   PROF="a;b;..."     bench.py argument sets, one rocprofv3 kernel-trace + stats run each
#   PROF_ENV="A=b"     environment of the PROF run
#   PMC="c1 c2;..."    PMC passes (one rocprofv3 run each) over PROF's bench args
#   PMC_ENV="A=b"      environment of the PMC runs
#   PRE="cmd"          a command run first (e.g. a probe binary), time-limited
# Every GPU step has its own time limit; the first failure ends the job.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/${OUT:-job}
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$PRE" ]; then
  timeout -k 10 120 bash -c "$PRE" > $O/pre.txt 2>&1 || { echo "PRE failed rc=$?"; tail -20 $O/pre.txt; exit 1; }
  cat $O/pre.txt
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread $TESTS > $O/pytest.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" $O/pytest.log | tail -${TEST_LINES:-40}
  tail -3 $O/pytest.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|error" $O/pytest.log | head -40; echo "pytest rc=$rc"; exit 1; }
fi
if [ -n "$BENCH" ]; then
  IFS=';' read -ra SETS <<< "$BENCH"
  i=0
  for a in "${SETS[@]}"; do
    i=$((i+1))
    # leading NAME=value words of an argument set are environment for that run
    envs=(); args=()
    for w in $a; do if [ ${#args[@]} -eq 0 ] && [[ "$w" == *=* ]]; then envs+=("$w"); else args+=("$w"); fi; done
    (for e in "${envs[@]}"; do export "$e"; done; timeout -k 10 200 python bench.py "${args[@]}") > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench '$a' failed"; tail -20 $O/bench_$i.err; exit 1; }
    echo "[$a] $(grep -h '^{' $O/bench_$i.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['config'].get('train_loss_mean', d['config'].get('train_loss_last')), d.get('eager',{}).get('ms_per_step'))")"
  done
fi
if [ -n "$PROF" ]; then
  # ";"-separated argument sets: prof (first), prof2, prof3, ...
  IFS=';' read -ra PSETS <<< "$PROF"
  j=0
  for a in "${PSETS[@]}"; do
    j=$((j+1)); d=prof; [ $j -gt 1 ] && d=prof$j
    (cd /tmp && { [ -z "$PROF_ENV" ] || export $PROF_ENV; } && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$d -o run --output-format csv -- python3 $R/bench.py $a > $O/$d.log 2>&1) \
      || { echo "prof '$a' failed"; tail -20 $O/$d.log; exit 1; }
    python3 $R/tools/prof_summary.py $O/$d > $O/kernel_summary_$j.txt 2>/dev/null || true
    f=$(ls $O/$d/*kernel_trace.csv 2>/dev/null | head -1)
    [ -n "$f" ] && python3 $R/tools/step_timeline.py $f > $O/step_timeline_$j.txt 2>/dev/null
    echo "== prof [$a]"; tail -${PROF_LINES:-30} $O/step_timeline_$j.txt 2>/dev/null
  done
  PROF=${PSETS[0]}
fi
if [ -n "$PMC" ]; then
  IFS=';' read -ra PS <<< "$PMC"
  i=0
  for c in "${PS[@]}"; do
    i=$((i+1))
    (cd /tmp && { [ -z "$PMC_ENV" ] || export $PMC_ENV; } && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/pmc$i -o run --output-format csv -- python3 $R/bench.py ${PROF:---steps 3 --warmup 1} --no-dist > $O/pmc$i.log 2>&1) \
      || { echo "pmc $i failed"; tail -5 $O/pmc$i.log; exit 1; }
    python3 $R/tools/pmc_summary.py $O/pmc$i/run_counter_collection.csv > $O/pmc$i.txt
  done
  cat $O/pmc*.txt | grep -A12 -E "${KPAT:-lenet|conv}" | head -${PMC_LINES:-80}
fi
exit 0
