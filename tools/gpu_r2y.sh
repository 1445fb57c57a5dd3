#!/bin/bash
# (1) LeNet-5 batch 163840 vs 131072; (2) PMC counters of the VGG-11 step (256-tile igemm kernels)
set -o pipefail
cd "$(dirname "$0")/.."
R=$PWD
O=$R/gpurun_out/r2y
mkdir -p $O
: > $O/ab.jsonl
for b in 131072 163840 131072 163840; do
  timeout -k 10 180 python bench.py --batch-per-gpu $b --steps 30 --warmup 5 >> $O/ab.jsonl 2>$O/err.log || { tail $O/err.log; exit 1; }
  echo "B=$b $(tail -1 $O/ab.jsonl | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['ms_per_step'], d['config']['train_loss_last'])")"
done
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set -d $O/pmc$i -o run --output-format csv -- python3 $R/bench.py --model vgg11 --batch-per-gpu 256 --steps 3 --warmup 1 --graph off > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $O/pmc1/run_counter_collection.csv $O/pmc2/run_counter_collection.csv > $O/pmc_summary.txt
grep -A14 "igemm_big_kernel<256, true, true\|igemm_dwbig_kernel<256" $O/pmc_summary.txt | head -40
