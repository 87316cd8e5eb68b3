# A/B of the length sort's workgroup floor (LVK_SORT_MIN_WGS) on C3 via offsets and the table bench.
# Variants first: tools/build_variant.sh old -DLVK_SORT_MIN_WGS=1; tools/build_variant.sh new -DLVK_SORT_MIN_WGS=256
set -o pipefail
R=$(pwd); O=gpurun_out/ab1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for rep in 1 2; do
for v in old new; do
  L=$R/leveldb-rs_amd/lib/variants/liblvgpu_$v.so
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$L timeout -k 10 200 python3 bench.py --workload c3 --api offsets --cpu-seconds 0 --traffic off > $O/${v}_c3o_$rep.json 2>$O/err || exit 1
  LVGPU_EXPERIMENT=1 LVGPU_LIB=$L timeout -k 10 200 python3 bench.py --table > $O/${v}_table_$rep.json 2>$O/err || exit 1
  python3 -c "import json; d=json.load(open('$O/${v}_c3o_$rep.json')); t=json.load(open('$O/${v}_table_$rep.json')); print('$v', d['value'], d['roofline']['frac'], 'seal', t['seal']['frac_of_8TBps'], 'verify', t['verify']['frac_of_8TBps'])"
done; done
