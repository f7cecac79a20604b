cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/sh8tl -o run --output-format csv -- python3 $R/bench.py --shard-of 8 --steps 30 --no-cpu-baseline --no-e2e --no-pmc > $R/gpurun_out/sh8tl.log 2>&1
