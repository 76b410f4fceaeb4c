set -u
export ABLATE_ONLY="full,pull0,pull1" ABLATE_EXTRA="pull0=-DGNCA_K1_PULL=0;pull1=-DGNCA_K1_PULL=1"
timeout -k 10 200 python tools/ablate.py run > gpurun_out/ab_pull_head.log 2>&1 || exit 1
ABLATE_CONFIG=c2 timeout -k 10 200 python tools/ablate.py run > gpurun_out/ab_pull_c2.log 2>&1 || exit 1
ABLATE_CONFIG=c3 timeout -k 10 200 python tools/ablate.py run > gpurun_out/ab_pull_c3.log 2>&1 || exit 1
ABLATE_PHASES=1 timeout -k 10 200 python tools/ablate.py run > gpurun_out/ab_pull_head_single.log 2>&1 || exit 1
