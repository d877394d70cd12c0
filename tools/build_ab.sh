# build an A/B variant of libured_hip.so into build_ab/<name>.so with extra -D flags
# usage: bash tools/build_ab.sh <name> -DFOO=0 ...
set -e
N=$1; shift
cd /root/repo
mkdir -p build_ab
P=387-u-red-unsupervised-3d-shape-retrieval-and-deformation-for-partial-point-clouds_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -mcode-object-version=5 \
  -Wno-unused-command-line-argument "$@" -I include $P/csrc/*.hip -o build_ab/$N.so
