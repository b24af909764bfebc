#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for W in 5 10 11; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup $W --no-cpu > gpurun_out/wu_$W.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/wu_$W.json')); print('warmup $W', d['ms_per_step'], d['roofline']['ms_per_launch'], d['kernels']['rhosum']['ms_per_launch'])"
done
