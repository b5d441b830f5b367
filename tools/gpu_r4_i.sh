#!/bin/bash
# GPU call (round 4): exhaustive v_log_f32 x*log2(x) accuracy, then the finisher's
# fp32 first pass with VALU terms (variants/vm*.so, MT_FIN_VMASK) A/B on the flagship.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result tools/probes/vlog_probe.hip -o /tmp/vlog_probe
timeout -k 10 60 /tmp/vlog_probe > gpurun_out/vlog_probe.log 2>&1
bash tools/gpu_ab_so.sh "$@"
