#!/bin/bash
# r04h: conv_il on the halo 3x3 too (per-layer A/B), the h2 / rank / ops GPU
# tests, and the C3 line with the new sweep and conv defaults
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 400 python -u tools/h2_cfg_sweep.py 1280 0,0i > $O/h2_cfg_il.txt 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_h2.py tests/test_gpu_rank.py tests/test_gpu_ops.py -m gpu -x -v -s --timeout 240 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log
tail -22 $O/h2_cfg_il.txt; tail -2 $O/tests.log; python -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['ms_per_step'],d['roofline']['frac_of_layer_floor'],d['roofline_by_kernel']['cosine_filter'])"
echo call-done
