# Interleaved A/B of library variants (tools/build_variant.sh) on offsets-API
# workloads and the table bench:  bash tools/ab_variants.sh OUT "vA vB" REPS
set -o pipefail
R=$(pwd); O=$1; vars=$2; reps=${3:-2}; mkdir -p $O
for rep in $(seq $reps); do
for v in $vars; do
  L=$R/leveldb-rs_amd/lib/variants/liblvgpu_$v.so
  line="$v"
  for w in c2 c4 c3; do
    LVGPU_EXPERIMENT=1 LVGPU_LIB=$L timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > $O/${v}_${w}_$rep.json 2>$O/err || exit 1
    line="$line $w $(python3 -c "import json; d=json.load(open('$O/${v}_${w}_$rep.json')); print(d['roofline']['frac'])")"
  done
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$L timeout -k 10 200 python3 bench.py --table > $O/${v}_table_$rep.json 2>$O/err || exit 1
  line="$line table $(python3 -c "import json; t=json.load(open('$O/${v}_table_$rep.json')); print(t['seal']['frac_of_8TBps'], t['verify']['frac_of_8TBps'])")"
  echo $line
done; done
