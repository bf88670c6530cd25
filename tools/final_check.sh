#!/bin/bash
# End-of-round evidence on one MI355X, from the tree as committed: STEP=tests -- full `pytest -m gpu`, smoke(), the
# driver's bench command (`python bench.py --gpus 1 --steps 20 --warmup 5`); STEP=prof -- rocprofv3 kernel stats of
# the headline bench and of the whole default bench, and the per-stage PMC passes (tools/pmc_all.sh) for MODELS.  Outputs: gpurun_out/final_*.
# Each GPU step has its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${STEP:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_gputests.log 2>&1 || { tail -30 gpurun_out/final_gputests.log; exit 1; }
  tail -1 gpurun_out/final_gputests.log
  timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
  tail -2 gpurun_out/final_smoke.log
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
  tail -1 gpurun_out/final_bench.json | cut -c1-600
else
  rm -rf gpurun_out/final_prof gpurun_out/final_prof_all
  # the headline alone (its kernels' averages are the bench line's per-launch figures), then the whole default
  # bench (the NAS / config-5 / train / eval512 legs' kernels; k_c12s there also averages the small batches)
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-extra-configs --steps 20 --warmup 5 > gpurun_out/final_prof.log 2>&1 || { tail -20 gpurun_out/final_prof.log; exit 1; }
  python tools/top_kernels.py "$(find gpurun_out/final_prof -name '*kernel_stats.csv' | head -1)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/final_prof_all -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/final_prof_all.log 2>&1 || { tail -20 gpurun_out/final_prof_all.log; exit 1; }
  MODELS="${MODELS:-hardnet wang2 wang3 wang4 c5}" timeout -k 10 900 bash tools/pmc_all.sh || exit 1
fi
echo done
