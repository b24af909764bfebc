#!/bin/bash
# Study variants of the block build (SPH_BEXP, k_blk_build) on the C2 1M rebuild, with the
# study library (make STUDY=1): per-phase cost by elimination.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
export SPH_HIP_LIB=$(pwd)/lammps-sph-multiphase_amd/libsph_hip_study.so
for e in 0 1 2 3 4; do
  echo -n "bexp $e: "; SPH_BEXP=$e timeout -k 10 150 python3 tools/build_sweep.py 100 10 || exit 1
done | tee gpurun_out/bexp_${1:-x}.log
