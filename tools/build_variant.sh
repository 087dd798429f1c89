#!/bin/bash
# Build an experimental variant of librmc.so next to the default one:
#   tools/build_variant.sh prof   -> tla-raft_amd/build_prof/librmc.so  (-DRMC_PHASE_PROF, tools/phase_prof.py)
#   tools/build_variant.sh w1     -> tla-raft_amd/build_w1/librmc.so    (n >= 4 expansion at 1 wave / SIMD)
# Select it with RMC_LIBRARY=<path> (raftmc.load_library).  Needs the default build (make -C tla-raft_amd).
set -e
cd "$(dirname "$0")/../tla-raft_amd"
FLAGS=""
for part in ${1//+/ }; do  # several specs joined by '+', e.g. fpb16+fw4
case "$part" in
  prof) FLAGS="$FLAGS -DRMC_PHASE_PROF" ;;
  # the sources as they are, beside the default build (an A/B of a source change: tools/ab_bench.sh)
  plain) ;;
  w1) FLAGS="$FLAGS -DRMC_WIDE_WAVES=1" ;;
  # the item-parallel split expansion: waves / SIMD its registers are cut for (e.g. iw6)
  iw*) FLAGS="$FLAGS -DRMC_ITEMS_WAVES=${part#iw}" ;;
  # the probe pass (k_hash_probe): waves / SIMD its registers are cut for (e.g. pw6)
  pw*) FLAGS="$FLAGS -DRMC_PROBE_WAVES=${part#pw}" ;;
  # ... its threads per block for n <= 3 (e.g. nt128; with pb32 the same items per thread)
  nt*) FLAGS="$FLAGS -DRMC_ITEMS_NT=${part#nt}" ;;
  # ... and its parents per batch (e.g. pb32)
  pb*) FLAGS="$FLAGS -DRMC_ITEMS_PB=${part#pb}" ;;
  # the fused item-parallel expansion's parents per batch (e.g. fpb8)
  fpb*) FLAGS="$FLAGS -DRMC_FUSED_PB=${part#fpb}" ;;
  # ... its commit's parents per block (e.g. fcpb8)
  fcpb*) FLAGS="$FLAGS -DRMC_FUSED_CPB=${part#fcpb}" ;;
  # ... and the waves / SIMD its registers are cut for (e.g. fw4)
  fw*) FLAGS="$FLAGS -DRMC_FUSED_WAVES=${part#fw}" ;;
  # n = 3 occupancy: expansion waves / SIMD, commit waves / SIMD, grid blocks / CU (e.g. n3w6c4g32)
  n3w*) X=${part#n3w}; W=${X%%c*}; X=${X#*c}; C=${X%%g*}; G=${X#*g}
        FLAGS="$FLAGS -DRMC_N3_WAVES=$W -DRMC_N3_COMMIT_WAVES=$C -DRMC_GRID_PER_CU=$G" ;;
  *) echo "usage: $0 prof|plain|w1|iw<W>|pw<W>|nt<T>|pb<P>|fpb<P>|fcpb<P>|fw<W>|n3w<W>c<C>g<G>[+...]" >&2; exit 2 ;;
esac
done
OUT=${VARIANT_DIR:-build_$1}  # (VARIANT_DIR: another directory for the same flags)
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -DRMC_WITH_RCCL $FLAGS -Iinclude -I../include -Icsrc \
  -c csrc/rmc_kernels.hip -o "$OUT/rmc_kernels.o"
$HIPCC --offload-arch=gfx950 -shared -fPIC -o "$OUT/librmc.so" "$OUT/rmc_kernels.o" build/rmc_engine.o build/rmc_cfg.o build/rmc_probe.o -lrccl
echo "$OUT/librmc.so"
