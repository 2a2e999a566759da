set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reuse
for v in a:"" b:"--graph-reuse" c:"" d:"--graph-reuse"; do
  tag=${v%%:*}; fl=${v#*:}
  timeout -k 10 240 python -m pertrenderer_amd.pose_opt --mode graph -np 30 $fl > gpurun_out/reuse/$tag.log 2>&1
  echo "$tag done"
done
