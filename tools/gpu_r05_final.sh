#!/bin/bash
# Round-5 evidence session: tools/gpu_round.sh (GPU suite, smoke, bench, rocprofv3 stats of the bench,
# PMC of the headline), then a trace + PMC of config 5's two kernels.
bash tools/gpu_round.sh || exit $?
bash tools/pmc.sh pmc_c5 python tools/config5_pmc_run.py > gpurun_out/pmc_c5.log 2>&1
rc=$?; echo "pmc c5 exit $rc"; tail -30 gpurun_out/pmc_c5.log
exit $rc
