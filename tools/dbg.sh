cd $GRAFT_REPO_ROOT
SPH_DEBUG=1 timeout -k 10 120 python3 tools/build_sweep.py 100 1 2>&1 | grep -E "sph\]|rebuild" | tail -3
