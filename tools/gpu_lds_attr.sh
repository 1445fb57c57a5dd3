#!/bin/bash
# LDS bank-conflict attribution per phase (MCC_ABLATE: 1 = no staging,
# 2 = no compute, 4 = no epilogue) for the LeNet-5 bench kernels.
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/ldsattr
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for a in ${ABL:-0 1 2 4}; do
  MCC_ABLATE=$a timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS -d $O/a$a -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 2 --no-dist > $O/a$a.log 2>&1 || { tail -5 $O/a$a.log; exit 1; }
  python $R/tools/pmc_summary.py $O/a$a/run_counter_collection.csv > $O/a$a.txt
done
python - "$O" <<'PY'
import sys, re, os
O = sys.argv[1]
def parse(f):
    d, k = {}, None
    for line in open(f):
        if not line.startswith(' '):
            k = line.strip(); d[k] = {}
        else:
            n, v = line.split(); d[k][n] = float(v)
    return d
runs = {a: parse(os.path.join(O, f'a{a}.txt')) for a in [x for x in os.environ.get('ABL', '0 1 2 4').split()]}
keys = [k for k in runs[next(iter(runs))] if 'conv' in k or 'fc_' in k or 'xent' in k or 'sgd' in k]
print(f"{'kernel':60s} " + ' '.join(f'abl{a}:lds/confl' for a in runs))
for k in keys:
    row = []
    for a, d in runs.items():
        v = d.get(k, {})
        row.append(f"{v.get('SQ_INSTS_LDS',0)/1e6:7.2f}/{v.get('SQ_LDS_BANK_CONFLICT',0)/1e6:7.2f}")
    print(f"{k[:60]:60s} " + '  '.join(row))
PY
