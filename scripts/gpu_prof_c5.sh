cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c5p1 -o run -- python3 $R/bench.py --config 5 --pipeline 1 --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/prof_c5p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_n2048 -o run -- python3 $R/bench.py --npkts 2048 --pipeline 1 --steps 20 --warmup 2 --no-cpu > $R/gpurun_out/prof_n2048.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trace_c5p1 -o run -- python3 $R/bench.py --config 5 --pipeline 1 --steps 4 --warmup 1 --no-cpu > $R/gpurun_out/trace_c5p1.log 2>&1 || exit 1
echo done
