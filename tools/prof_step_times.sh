#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/st; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o st -- python3 $R/tools/step_times.py 100 22 > $O/st.log 2>&1 || exit 1
cd $R && python3 tools/rebuild_compare.py "$(find $O/prof -name '*kernel_trace.csv' | head -1)"
