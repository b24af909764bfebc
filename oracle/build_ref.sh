#!/bin/bash
# Build oracle/_ref/libsph_ref.so: the reference's own USER-SPH compute code (plus the
# neighbor builders and the Pair/Neighbor/Comm/Memory base classes it runs on), compiled
# straight from the sources under /root/reference/src with g++, no reference build
# system, no generated headers, nothing copied into this repo.  Driven by
# oracle/ref_harness.cpp.  TEST INFRASTRUCTURE ONLY (parity pinning + golden fixtures).
#
# Translation units that need the generated style_*.h headers (atom.cpp, domain.cpp,
# force.cpp, update.cpp, lammps.cpp, modify.cpp, ...) are deliberately NOT compiled; the
# shared object is linked with those symbols unresolved and the harness never calls them.
set -euo pipefail
REF=${REF:-/root/reference/src}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
# VARIANT=fma: the same sources built for an FMA machine (-mfma, GCC contracting a*b+c as it
# does by default there) into oracle/_ref_fma/libsph_ref.so -- how far the reference's own
# results move between two legitimate builds (tools/fma_build_shift.py); not the oracle
# VARIANT=fastmath: the reference's own fast-math recipe (src/MAKE/Makefile.mingw64-cross:10-11)
# into oracle/_ref_fastmath/libsph_ref.so
if [ "${VARIANT:-}" = "fma" ]; then OUT=$HERE/_ref_fma; fi
if [ "${VARIANT:-}" = "fastmath" ]; then OUT=$HERE/_ref_fastmath; fi
OBJ=$OUT/obj
mkdir -p "$OBJ"
if [ ! -d "$REF" ]; then
  echo "build_ref.sh: $REF not present (GPU box?) -- skipping reference oracle build" >&2
  exit 0
fi

CORE="pair.cpp memory.cpp error.cpp comm.cpp comm_brick.cpp neighbor.cpp neigh_full.cpp
      neigh_half_bin.cpp neigh_half_nsq.cpp neigh_half_multi.cpp neigh_half_respa.cpp
      neigh_derive.cpp neigh_stencil.cpp neigh_list.cpp neigh_request.cpp neigh_bond.cpp
      neigh_gran.cpp neigh_full.cpp neigh_respa.cpp atom_vec.cpp citeme.cpp fix.cpp
      group.cpp random_park.cpp region.cpp region_block.cpp"
SPH="atom_vec_meso.cpp atom_vec_meso_multiphase.cpp pair_sph_rhosum.cpp
     pair_sph_taitwater.cpp pair_sph_taitwater_morris.cpp pair_sph_heatconduction.cpp
     pair_sph_rhosum_multiphase.cpp pair_sph_taitwater_multiphase.cpp
     pair_sph_heatconduction_phasechange.cpp pair_sph_colorgradient.cpp
     pair_sph_surfacetension.cpp sph_kernel_quintic.cpp sph_energy_equation.cpp
     fix_meso.cpp fix_meso_stationary.cpp fix_phase_change.cpp"

# the reference's own serial build: g++ -O3 at the compiler's default C++ dialect (src/MAKE/
# Makefile.serial:9-10); the dialect matters -- under C++98 pow(double,int) is __builtin_powi
CXXFLAGS="-O3 -fPIC -w -DLAMMPS_SMALLBIG -I$REF -I$REF/USER-SPH -I$REF/STUBS"
if [ "${VARIANT:-}" = "fma" ]; then CXXFLAGS="$CXXFLAGS -mfma -ffp-contract=fast"; fi
if [ "${VARIANT:-}" = "fastmath" ]; then
  CXXFLAGS="$CXXFLAGS -march=core2 -mtune=core2 -msse2 -ffast-math -fstrict-aliasing"
fi
objs=()
compile() {  # src obj
  if [ ! -f "$2" ] || [ "$1" -nt "$2" ]; then g++ $CXXFLAGS -c "$1" -o "$2"; fi
}
pids=()
for f in $(echo $CORE | tr ' ' '\n' | sort -u); do
  [ -f "$REF/$f" ] || continue
  o=$OBJ/${f%.cpp}.o; objs+=("$o"); compile "$REF/$f" "$o" & pids+=($!)
done
for f in $SPH; do
  o=$OBJ/sph_${f%.cpp}.o; objs+=("$o"); compile "$REF/USER-SPH/$f" "$o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
gcc -O2 -fPIC -w -I$REF/STUBS -c "$REF/STUBS/mpi.c" -o "$OBJ/mpi_stubs.o"
g++ $CXXFLAGS -c "$HERE/ref_harness.cpp" -o "$OBJ/ref_harness.o"
# Python's ctypes dlopen()s with RTLD_NOW, so references into the translation units we
# do not build must not be fatal at load time: mark exactly those LAMMPS_NS symbols that
# are referenced but defined nowhere in our objects as weak (they resolve to null and are
# never called by the harness).
WEAK=$OBJ/weak; mkdir -p "$WEAK"; wobjs=()
allo=("${objs[@]}" "$OBJ/ref_harness.o")
nm -u "${allo[@]}" 2>/dev/null | awk 'NF==2 && $1=="U"{print $2}' | sort -u > "$OBJ/undef.txt"
nm --defined-only "${allo[@]}" 2>/dev/null | awk 'NF==3{print $3}' | sort -u > "$OBJ/def.txt"
comm -23 "$OBJ/undef.txt" "$OBJ/def.txt" | grep '9LAMMPS_NS' > "$OBJ/weaken.txt" || true
for o in "${allo[@]}"; do
  w=$WEAK/$(basename "$o"); objcopy --weaken-symbols="$OBJ/weaken.txt" "$o" "$w"; wobjs+=("$w")
done
g++ -shared -o "$OUT/libsph_ref.so" "${wobjs[@]}" "$OBJ/mpi_stubs.o"
echo "built $OUT/libsph_ref.so"

# libsph_shim.so: the same reference objects with the drop-in style classes of this repo
# (lammps-sph-multiphase_amd/lammps/*.cpp: sph/<style>/hip, fix phase_change/hip) linked
# in, as LAMMPS would link them, and the harness built with -DSPH_SHIM (entry points
# shim_*): the classes run their compute()/pre_exchange() through libsph_hip.so on the
# harness-filled universe.  Needs the product library built first (make -C the package).
PKG=$HERE/../lammps-sph-multiphase_amd
if [ -f "$PKG/libsph_hip.so" ] && [ -z "${VARIANT:-}" ]; then
  SHIMF="-I$PKG/lammps -I$HERE/../include"
  sobjs=()
  for f in pair_sph_hip fix_phase_change_hip; do
    o=$OBJ/shim_$f.o; sobjs+=("$o")
    if [ ! -f "$o" ] || [ "$PKG/lammps/$f.cpp" -nt "$o" ] || [ "$PKG/lammps/$f.h" -nt "$o" ] ||
       [ "$HERE/../include/sph_hip.h" -nt "$o" ]; then
      g++ $CXXFLAGS $SHIMF -c "$PKG/lammps/$f.cpp" -o "$o"
    fi
  done
  g++ $CXXFLAGS $SHIMF -DSPH_SHIM -c "$HERE/ref_harness.cpp" -o "$OBJ/shim_harness.o"
  sall=("${objs[@]}" "${sobjs[@]}" "$OBJ/shim_harness.o")
  nm -u "${sall[@]}" 2>/dev/null | awk 'NF==2 && $1=="U"{print $2}' | sort -u > "$OBJ/sundef.txt"
  nm --defined-only "${sall[@]}" 2>/dev/null | awk 'NF==3{print $3}' | sort -u > "$OBJ/sdef.txt"
  comm -23 "$OBJ/sundef.txt" "$OBJ/sdef.txt" | grep '9LAMMPS_NS' > "$OBJ/sweaken.txt" || true
  SW=$OBJ/sweak; mkdir -p "$SW"; swobjs=()
  for o in "${sall[@]}"; do
    w=$SW/$(basename "$o"); objcopy --weaken-symbols="$OBJ/sweaken.txt" "$o" "$w"; swobjs+=("$w")
  done
  g++ -shared -o "$OUT/libsph_shim.so" "${swobjs[@]}" "$OBJ/mpi_stubs.o" -L"$PKG" -lsph_hip \
      -Wl,-rpath,'$ORIGIN/../../lammps-sph-multiphase_amd'
  echo "built $OUT/libsph_shim.so"
fi
