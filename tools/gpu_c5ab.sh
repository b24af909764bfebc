#!/bin/bash
# C5 engine tests, then C5 bench lines of library builds / env settings:
# tools/gpu_c5ab.sh SPEC ... (SPEC as tools/gpu_ab.sh)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out/c5ab
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_c5_engine.py tests/test_c5_bricks.py tests/test_gpu_multiphase.py -m gpu -q \
  --timeout 240 --timeout-method thread > gpurun_out/c5ab/tests.log 2>&1 || { tail -30 gpurun_out/c5ab/tests.log; exit 1; }
tail -2 gpurun_out/c5ab/tests.log
fi
ARGS=${AB_ARGS:---workload c5 --steps 10 --warmup 3 --no-cpu}
for SPEC in "$@"; do
  IFS=: read -r L ENVS <<< "$SPEC"
  P=lammps-sph-multiphase_amd/$L; [ "$L" = prod ] && P=lammps-sph-multiphase_amd/libsph_hip.so
  TAG=$(echo "$SPEC" | tr ':=/' '___')
  env ${ENVS//:/ } SPH_HIP_LIB=$(pwd)/$P timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/c5ab/$TAG.json 2> gpurun_out/c5ab/$TAG.err || { tail -3 gpurun_out/c5ab/$TAG.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/c5ab/$TAG.json')); k=d.get('kernels',{})
print('%-40s value %.4g ms/step %.3f' % ('$SPEC', d['value'], d['ms_per_step']), {a: (round(b,3) if isinstance(b,float) else b) for a,b in k.items() if not isinstance(b,(dict,str))}, k.get(next(iter(k)),{}))"
done
