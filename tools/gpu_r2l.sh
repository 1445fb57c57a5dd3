#!/bin/bash
# u8 first-layer dword-run staging: tests + VGG A/B (MCC_U8_RUNS) + kernel summary
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_igemm.py tests/test_gpu_engine.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 0 1; do
  MCC_U8_RUNS=$r timeout -k 10 180 python bench.py --model vgg11 --batch-per-gpu 256 --steps 10 --warmup 3 > $O/vgg_$r.json 2>$O/vgg.err || { tail $O/vgg.err; exit 1; }
  echo "runs=$r $(tail -1 $O/vgg_$r.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_vgg -o run --output-format csv -- python3 $R/bench.py --model vgg11 --batch-per-gpu 256 --steps 8 --warmup 2 --graph off > $O/prof_vgg.log 2>&1 || { tail $O/prof_vgg.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof_vgg > $O/vgg_summary.txt 2>&1
python3 $R/tools/step_timeline.py $O/prof_vgg/run_kernel_trace.csv > $O/vgg_timeline.txt
head -14 $O/vgg_summary.txt
