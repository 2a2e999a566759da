# round 4: RCCL one-rank runs of bench.py's distributed path and of exact mode's collectives
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rccl.py tests/test_gpu_exact_shards.py > gpurun_out/tests_r4w.log 2>&1
rc=$?; tail -n 12 gpurun_out/tests_r4w.log; exit $rc
