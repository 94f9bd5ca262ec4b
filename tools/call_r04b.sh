#!/bin/bash
# r04b: fetch-ceiling microbenchmark, trunk/rank overlap probe, sweep-order A/B,
# pipelined vs serial C3 bench, changed GPU tests
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 120 ./tools/fetch_ceiling 5 > $O/fetch_ceiling.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/hbm_pattern > $O/hbm_pattern.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/overlap_probe.py > $O/overlap.txt 2>&1 || exit 1
PF_KEY=sweep_order PF_CFGS="0 2 4" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/sweep_order_ab.txt 2>&1 || exit 1
PF_QKIND=corr PF_KEY=sweep_order PF_CFGS="0 2 4" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/sweep_order_ab_corr.txt 2>&1 || exit 1
PF_KEY=sweep_pf PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/sweep_pf_ab.txt 2>&1 || exit 1
PF_QKIND=corr PF_KEY=sweep_pf PF_CFGS="0 1" timeout -k 10 300 python -u tools/prefilter_ab.py > $O/sweep_pf_ab_corr.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --pipeline 1 > $O/c3_pipe.json 2> $O/c3_pipe.log || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --pipeline 0 > $O/c3_serial.json 2> $O/c3_serial.log || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_vit.py tests/test_gpu_c2.py tests/test_gpu_e2e_lowp.py tests/test_gpu_rank.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -3 $O/tests.log
echo call-done
