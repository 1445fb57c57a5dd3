#!/bin/bash
# Build the Python module of a git ref into build/ab_<name>/ for same-box A/B
# runs:  tools/ab_build.sh HEAD old  ->  python build/ab_old/bench.py ...
set -e
ref=${1:-HEAD}; name=${2:-old}
cd "$(dirname "$0")/.."
src=build/ab_src_$name; dst=build/ab_$name
rm -rf $src $dst; mkdir -p $src $dst
git archive $ref | tar -x -C $src
make -C $src -j8 module >/dev/null
cp -r $src/mpi_cuda_cnn_amd $dst/
cp $src/bench.py $dst/
find $dst -name __pycache__ -prune -exec rm -rf {} \;
rm -rf $src
echo "built $ref -> $dst"
