# rocprofv3 kernel trace + stats, then separate PMC passes (FETCH_SIZE, WRITE_SIZE)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 990 --warmup 10 --no-cpu-baseline > gpurun_out/prof/bench_trace.log 2>&1 && echo TRACE_OK && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-profile > gpurun_out/prof/bench_fetch.log 2>&1 && echo FETCH_OK && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-profile > gpurun_out/prof/bench_write.log 2>&1 && echo WRITE_OK
ls -R gpurun_out/prof | head -40
