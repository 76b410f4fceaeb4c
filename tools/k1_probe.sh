#!/bin/bash
# Register / ISA study of one K1 instance without building the library:
#   tools/k1_probe.sh "<template args>" [extra hipcc flags]   e.g. tools/k1_probe.sh "24,36,4,4,8,0,false" -DGNCA_K1_SPLIT_NT=768
#   K=gnca_k2_finalize tools/k1_probe.sh "4,true,2,false"   (another kernel template defined before the host code)
# prints the kernel-resource-usage remark; the ISA goes to /tmp/k1probe/*.s
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
ARGS=$1; shift
mkdir -p /tmp/k1probe
cat > /tmp/k1probe/probe.hip <<EOT
#define GNCA_K1_PROBE 1
#include "$ROOT/graph_neural_cellular_automata_amd/csrc/gnca_step.hip"
template __global__ void ${K:-gnca_k1_split}<$ARGS>(const ${KA:-K1Args});
}  // namespace gnca (left open by the GNCA_K1_PROBE cut)
EOT
cd /tmp/k1probe
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -I"$ROOT/include" --cuda-device-only -S \
  "$@" probe.hip -o probe.s -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "VGPRs|AGPRs|Spill|Occupancy|ScratchSize|LDS" | sed 's/.*remark: //'
