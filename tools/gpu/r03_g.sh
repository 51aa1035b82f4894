# round 3, call g: op-level attribution of one fp16 training step (torch.profiler), then a bench line with the
# gather probe
set -o pipefail
R=$GRAFT_REPO_ROOT
cd "$R" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u tools/op_profile.py --attribute --rows 60 > gpurun_out/op_profile_fp16.txt 2>&1 && echo "[g] profile ok" && \
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-modes > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err && echo "[g] bench ok"
