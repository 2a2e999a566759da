# round 4: rast_fwd occupancy x slices (4 waves/SIMD build with 8 slices: all heavy 4x2 tiles resident?)
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
bash tools/gpu.sh sweep r4j cfg2 "base|PR_X=0|" "sl8|PR_RAST_SLICES=8|" "wpe4|PR_X=0|libpertrender_wpe4" \
  "wpe4sl8|PR_RAST_SLICES=8|libpertrender_wpe4" "base2|PR_X=0|" "wpe4sl8b|PR_RAST_SLICES=8|libpertrender_wpe4" || exit 1
bash tools/gpu.sh sweep r4je eval "base|PR_X=0|" "wpe4sl8|PR_RAST_SLICES=8|libpertrender_wpe4" || exit 1
