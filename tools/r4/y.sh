# round 4: blend per-block phase profile at cfg 2 (current code)
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 200 python tools/blend_prof.py > gpurun_out/blend_prof_r4.txt 2>&1
rc=$?; cat gpurun_out/blend_prof_r4.txt | grep -v amdgpu.ids; exit $rc
