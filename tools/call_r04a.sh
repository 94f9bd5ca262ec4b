set -o pipefail
O=gpurun_out/r04a; mkdir -p $O
bash tools/rc_quick.sh r04a && \
timeout -k 10 300 python -u tools/chunk_probe.py > $O/chunk_probe.txt 2>&1 && \
bash tools/resid_pmc.sh gpurun_out/r04a/pmc > $O/pmc.log 2>&1 && \
timeout -k 10 400 python -u bench.py > $O/c3.json 2> $O/c3.log && echo call-done
