# Interleaved bench.py --sweep under library variants: bash tools/ab_sweep.sh OUT "vA vB" REPS
set -o pipefail
R=$(pwd); O=$1; vars=$2; reps=${3:-1}; mkdir -p $O
for rep in $(seq $reps); do
for v in $vars; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$R/leveldb-rs_amd/lib/variants/liblvgpu_$v.so timeout -k 10 300 python3 bench.py --sweep > $O/${v}_sweep_$rep.json 2>$O/err || exit 1
  python3 -c "
import json; d=json.load(open('$O/${v}_sweep_$rep.json'))
rows=d['results']
print('$v', [(r['block_KiB'], r['strided']['frac_of_8TBps'] if isinstance(r.get('strided'),dict) else r.get('strided'), r['offsets']['frac_of_8TBps'] if isinstance(r.get('offsets'),dict) else r.get('offsets')) for r in rows])" || { cat $O/${v}_sweep_$rep.json | head -c 600; }
done; done
