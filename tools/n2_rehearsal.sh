# 2-rank bench rehearsal on a 1-GPU box: both ranks share cuda:0 (gloo for the
# collectives, since RCCL refuses two ranks on one device); checks the N>1 code
# path of every workload end to end.  Never used for reported numbers.
set -o pipefail
O=gpurun_out/n2
mkdir -p $O
export RR_DIST_BACKEND=gloo
timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 > $O/c3.json 2> $O/c3.err && \
timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --workload c5 > $O/c5.json 2> $O/c5.err && \
timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --workload c4 > $O/c4.json 2> $O/c4.err && \
echo all-done
