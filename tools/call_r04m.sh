#!/bin/bash
# r04m: the ViT LayerNorm fold -- its tests, the C4 e2e test, an interleaved
# A/B on the C4 embed, and the C4 line
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_vit.py tests/test_gpu_lowp.py tests/test_gpu_e2e_lowp.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
grep -E "fold|C4 bf16" $O/tests.log; tail -1 $O/tests.log
E2E_WORKLOAD=c4 E2E_EMBED="ln_fold=0 ln_fold=1" timeout -k 10 400 python -u tools/e2e_ab.py 1280 5 > $O/e2e_c4_fold.txt 2>&1 && grep -v amdgpu.ids $O/e2e_c4_fold.txt && \
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline > $O/c4.json 2> $O/c4.log && python -c "import json;d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:(v.get('ms_per_step'),v.get('frac')) for k,v in d['roofline_by_kernel'].items()})"
echo call-done
