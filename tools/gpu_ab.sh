#!/bin/bash
# A/B of library builds / env settings on the C2 bench: tools/gpu_ab.sh SPEC ... with SPEC =
# lib[:VAR=val[:VAR=val]] (lib relative to the package dir; "prod" = libsph_hip.so).  Prints
# value, force/rhosum ms per launch, neighbour build ms per rebuild for each.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out/ab
ARGS=${AB_ARGS:---steps 100 --warmup 20 --no-cpu}
for SPEC in "$@"; do
  IFS=: read -r L ENVS <<< "$SPEC"
  P=lammps-sph-multiphase_amd/$L; [ "$L" = prod ] && P=lammps-sph-multiphase_amd/libsph_hip.so
  TAG=$(echo "$SPEC" | tr ':=/' '___')
  env ${ENVS//:/ } SPH_HIP_LIB=$(pwd)/$P timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/ab/$TAG.json 2> gpurun_out/ab/$TAG.err || { tail -3 gpurun_out/ab/$TAG.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab/$TAG.json')); k=d.get('kernels',{})
print('%-40s value %.4g ms/step %.4f force %.4f rho %.4f build %s' % ('$SPEC', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], k.get('rhosum',{}).get('ms_per_launch',0), k.get('neighbor_build_ms')))"
done
