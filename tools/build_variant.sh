#!/bin/bash
# A kernel-experiment build of libgfpl_hip.so from the current sources with extra compiler
# flags (e.g. -DLSD_SORT_CAP=512), into OUTDIR beside a copy of libgfpl_synth.so; load it with
# GFPL_LIB_DIR=OUTDIR (tools/ab_bench.sh).  CPU-side (hipcc cross-compiles for gfx950).
# usage: tools/build_variant.sh OUTDIR [flags...]
set -e
out=$1; shift
cd "$(dirname "$0")/.."
mkdir -p "$out"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Wall -Wno-unused-result \
    -Iinclude "$@" gf-pl-slam_amd/csrc/*.hip gf-pl-slam_amd/csrc/*.cpp -o "$out/libgfpl_hip.so"
cp gf-pl-slam_amd/lib/libgfpl_synth.so "$out/"
echo "$out: $*" > "$out/FLAGS"
