# A/B of the sort's workgroup floor on C2/C4 (1M buffers): variants new (-DLVK_SORT_MIN_WGS=256) and w1024 (=1024),
# built with tools/build_variant.sh
set -o pipefail
R=$(pwd); O=gpurun_out/ab2; mkdir -p $O
for rep in 1 2; do
for v in new w1024; do
  L=$R/leveldb-rs_amd/lib/variants/liblvgpu_$v.so
  for w in c2 c4; do
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$L timeout -k 10 200 python3 bench.py --workload $w --api offsets --cpu-seconds 0 --traffic off > $O/${v}_${w}_$rep.json 2>$O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/${v}_${w}_$rep.json')); print('$v $w', d['value'], d['roofline']['frac'])"
  done
done; done
