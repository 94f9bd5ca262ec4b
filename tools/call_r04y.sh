#!/bin/bash
# r04y: the final tree -- the whole -m gpu suite + smoke, the C3 and C4 lines
set -o pipefail
O=gpurun_out/r04y; mkdir -p $O
bash tools/rc_quick.sh r04y || { grep -E "FAILED|Error" $O/gpu_tests.log | head; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log && \
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu-baseline > $O/c4.json 2> $O/c4.log
for f in c3 c4; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],{k:(v.get('ms_per_step'),v.get('frac')) for k,v in d['roofline_by_kernel'].items()})"; done
echo call-done
