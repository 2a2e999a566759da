# smoke + GPU tests + bench, then a kernel trace of the eager step
set -u
R="$GRAFT_REPO_ROOT"; TAG="${1:-qk}"
bash "$R/tools/gpu_quick.sh" "$TAG" || exit $?
bash "$R/tools/gpu_ktrace.sh" "kt_$TAG"
