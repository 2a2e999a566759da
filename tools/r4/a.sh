# round 4 (re-entry): full GPU suite at HEAD, one bench line, and a kernel trace of 20 graph steps (step timeline)
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
bash tools/gpu.sh tests r4a || exit 1
bash tools/gpu.sh bench r4a --no-dense || exit 1
bash tools/gpu.sh prof r4a --steps 20 --warmup 5 --no-cpu-baseline --no-dense || exit 1
