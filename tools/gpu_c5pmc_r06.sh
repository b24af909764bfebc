set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r06/c5final; mkdir -p $O
META="world=1 edge=159 path=0 steps=5 warmup=2 commit=d69e714" timeout -k 10 900 tools/pmc_traffic.sh $O/pmc_c5 --workload c5 --steps 5 --warmup 2 --no-cpu
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o c5 -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/bench_c5_prof.json 2> $O/prof_c5.err
echo done
