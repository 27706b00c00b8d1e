# usage: bash tools/asan_host.sh [pytest -k expr]: the RMSD mode's host C extension (csrc/rmsdkey.c,
# csrc/frepr.cpp) built with AddressSanitizer + UndefinedBehaviorSanitizer and run under the CPU
# host-path tests (build container only: host code, no GPU)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
OUT=/tmp/geobpe_asan
mkdir -p $OUT
PYINC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -g -O1"
g++ $SAN -fPIC -std=c++17 -c pt-bpe_amd/csrc/frepr.cpp -o $OUT/frepr.o || exit 1
gcc $SAN -shared -fPIC -I$PYINC pt-bpe_amd/csrc/rmsdkey.c $OUT/frepr.o -lstdc++ -o $OUT/_rmsdkey.so || exit 1
K=${1:-"host or pair_key or set_geo or key_float or memo or prio"}
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
GEOBPE_RMSDKEY=$OUT/_rmsdkey.so \
  python3 -m pytest tests/test_rmsd_mode.py tests/test_glue.py -m "not gpu" -q -x -k "$K" -p no:cacheprovider
