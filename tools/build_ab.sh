#!/bin/bash
# Whole-library A/B variants for tools/ab_c5.sh: fedscale_amd/ab/libfedagg_<name>.so from the current sources with
# extra -D flags (each carries its build id and defs: the loader checks it against the tree, buildinfo.py).
#   bash tools/build_ab.sh base ""  maxk2048 "-DQF_MAXK=2048"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $ROOT/fedscale_amd/ab
cd $ROOT
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  python3 -m fedscale_amd.buildinfo --out $ROOT/fedscale_amd/ab/libfedagg_$name.so --defs="$defs" --force
done
