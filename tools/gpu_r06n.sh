#!/bin/bash
# counters of the s2d stem kernels (fwd, wgrad)
set -o pipefail
R=$GRAFT_REPO_ROOT
bash tools/pmc_conv.sh stem fwd > /dev/null 2>&1 || exit 21
bash tools/pmc_conv.sh stem wgrad > /dev/null 2>&1 || exit 22
python3 tools/pmc_report.py gpurun_out/pmc_stem_fwd
python3 tools/pmc_report.py gpurun_out/pmc_stem_wgrad
