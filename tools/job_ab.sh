#!/bin/bash
# r04 job: GT-first sweep classes (valid allele = '.'..'9' but '/', one bcnt with accumulator per
# count): the AF tests, then GT:AD:DP A/B against the previous build (build_gfprev)
bash gpu_job.sh test tests/test_gpu_af.py tests/test_gpu_af_fused.py tests/test_gpu_cli.py || exit $?
bash gpu_job.sh ab gtadp build_gfprev/libvcfx_gpu.so 3 --steps 20 --format gt:ad:dp || exit $?
