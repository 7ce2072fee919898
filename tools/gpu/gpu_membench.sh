set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out /tmp/mb
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o /tmp/mb/membench || exit 1
timeout -k 10 300 /tmp/mb/membench 1073741824 > gpurun_out/membench.log 2>&1; rc=$?
cat gpurun_out/membench.log; exit $rc
