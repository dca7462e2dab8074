#!/bin/bash
# Build a measurement variant of libuampath.so (compile-time knobs) beside the product build:
#   tools/build_variant.sh <name> "<hipcc flags>"   ->  build/variants/libuampath_<name>.so
# Load it with UAM_LIB_PATH (uam_path_planning_amd/_lib.py).  Product code never loads these.
set -eu
cd "$(dirname "$0")/.."
name=$1
flags=${2:-}
mkdir -p build/variants
c=uam_path_planning_amd/csrc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 -Wall \
    $flags -o build/variants/libuampath_$name.so $c/uampath.hip $c/polyproc.cpp $c/tiles.cpp -lz
echo build/variants/libuampath_$name.so
