# 4-rank bench rehearsal on a 1-GPU box (all ranks on cuda:0, gloo collectives):
# exercises the all-gather / all-to-all / merge and the alpha-QE row exchange at
# world 4.  Never used for reported numbers.
set -o pipefail
O=gpurun_out/n4
mkdir -p $O
export RR_DIST_BACKEND=gloo
timeout -k 10 500 python -u bench.py --gpus 4 --steps 2 --warmup 1 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 500 python -u bench.py --gpus 4 --steps 2 --warmup 1 --workload c5 > $O/c5.json 2> $O/c5.err && \
echo all-done
