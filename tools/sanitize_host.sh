#!/bin/bash
# CPU suite against the host code built with AddressSanitizer + UBSan
# (leveldb-rs_amd `make sanitize`; GPU kernels are not instrumented: GPU ASan
# is unavailable on this pool).  Runs here, no GPU needed.
set -eo pipefail
root=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$root/leveldb-rs_amd" sanitize > /dev/null
export LVGPU_EXPERIMENT=1
export LVGPU_LIB="$root/leveldb-rs_amd/lib/variants/liblvgpu_asan.so"
export LD_PRELOAD="$(gcc -print-file-name=libasan.so)"
export ASAN_OPTIONS=detect_leaks=0
export PYTHONPATH="$root/leveldb-rs_amd${PYTHONPATH:+:$PYTHONPATH}"
python3 -c "import lvgpu, sys; lvgpu.lib(); m = open('/proc/self/maps').read(); sys.exit(0 if 'liblvgpu_asan.so' in m and 'libasan' in m else 'sanitized library not loaded')"
cd "$root" && python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
