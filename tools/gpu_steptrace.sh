#!/bin/bash
# Kernel timeline of one LeNet-5 bench step WITH the RCCL process group (1 rank)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD; O=$R/gpurun_out/steptrace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/run -o run --output-format csv -- python $R/bench.py --steps 10 --warmup 3 ${ARGS} > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
python - $O <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + '/run/*kernel_trace.csv')[0]
rows = list(csv.DictReader(open(f)))
ks = sorted([(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], r['Queue_Id']) for r in rows])
idx = [i for i, k in enumerate(ks) if 'sgd_pack' in k[2]]
a, b = idx[-3], idx[-2]
t0 = ks[a][1]
for k in ks[a + 1:b + 1]:
    print(f"{(k[0]-t0)/1000:8.1f} {(k[1]-k[0])/1000:7.1f} q{k[3]:>2} {k[2][:80]}")
print("step", (ks[b][1] - ks[a][1]) / 1000, "us")
PY
