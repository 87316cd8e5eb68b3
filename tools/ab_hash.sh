# Interleaved A/B of hash-kernel variants on bench.py --hash:
#   SRC=hash tools/build_variant.sh p2 -DLVH_PIPE2=1; SRC=hash tools/build_variant.sh p1 -DLVH_PIPE2=0
#   bash tools/ab_hash.sh OUT "p2 p1" REPS
set -o pipefail
R=$(pwd); O=$1; vars=$2; reps=${3:-2}; mkdir -p $O
for rep in $(seq $reps); do
for v in $vars; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$R/leveldb-rs_amd/lib/variants/liblvgpu_$v.so timeout -k 10 200 python3 bench.py --hash > $O/${v}_hash_$rep.json 2>$O/err || exit 1
  echo "$v $(python3 -c "import json; d=json.load(open('$O/${v}_hash_$rep.json')); print(d['value'], d['frac_of_8TBps'])")"
done; done
