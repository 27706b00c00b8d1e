# usage: bash tools/ab_build.sh <name> "<-D flags>"  -> pt-bpe_amd/geobpe/ab_<name>.so (kernel A/B variants; CPU side)
# the same sources as geobpe/build.py (geobpe.hip) with extra -D flags
set -e
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -Wall -Wno-unused-result \
  -Wno-unused-value -Wno-unused-function $2 pt-bpe_amd/csrc/geobpe.hip -o pt-bpe_amd/geobpe/ab_$1.so
echo pt-bpe_amd/geobpe/ab_$1.so
