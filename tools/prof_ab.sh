#!/bin/bash
# rocprofv3 kernel stats of the C2 bench for several library builds: tools/prof_ab.sh LIB...
# (LIB relative to the package dir; "prod" = libsph_hip.so).  Prints the top kernels of each.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
ARGS=${AB_ARGS:---steps 40 --warmup 5 --no-cpu}
for L in "$@"; do
  P=lammps-sph-multiphase_amd/$L; [ "$L" = prod ] && P=lammps-sph-multiphase_amd/libsph_hip.so
  D=gpurun_out/pab/$(basename "$L" .so)
  SPH_HIP_LIB=$(pwd)/$P bash tools/prof_bench.sh "$D" $ARGS || exit 1
  echo "== $L $(python3 -c "import json;d=json.load(open('$D/bench.json'));print('value %.4g ms/step %.4f'%(d['value'],d['ms_per_step']))")"
  python3 tools/kstats.py "$D/bench_kernel_stats.csv" ${TOP:-6}
done
