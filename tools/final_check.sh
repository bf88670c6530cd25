# End-of-session check on one MI355X: GPU tests, smoke, bench lines (config 2, config 5) and the
# rocprofv3 kernel stats of the config-2 bench.  Output: gpurun_out/final_*
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gputests.log 2>&1 || { tail -20 gpurun_out/final_gputests.log; exit 1; }
tail -1 gpurun_out/final_gputests.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
tail -1 gpurun_out/final_bench.json
timeout -k 10 300 python bench.py --config 5 > gpurun_out/final_bench_c5.json 2> gpurun_out/final_bench_c5.err || { tail -20 gpurun_out/final_bench_c5.err; exit 1; }
tail -1 gpurun_out/final_bench_c5.json
rm -rf gpurun_out/final_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
echo done
