# Round 6: the bench's checked exchange (one-rank torchrun, config 4, --exchange ipc)
# and the long kernel's per-phase timeline at config 3 (timeline variant build).
set -o pipefail
OUT=gpurun_out/${TAG:-r6tl3}
mkdir -p $OUT
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29655 bench.py --gpus 1 --steps 40 --warmup 1 --config cfg4 --exchange ipc --no-side \
  --no-cpu-baseline > $OUT/bench_cfg4_ipc.json 2> $OUT/bench_cfg4_ipc.log || exit 1
python3 -c "import json; r=json.load(open('$OUT/bench_cfg4_ipc.json')); print(r['exchange'], r['config']['parallelism'], round(r['ms_per_step']*1e3,2))"
GS_TL_LIB=libgibbs_hip_tl.so timeout -k 10 300 python -u tools/timeline.py ${TLCFGS:-cfg3:init} > $OUT/tl.json 2> $OUT/tl.err || { tail -5 $OUT/tl.err; exit 1; }
python3 - $OUT/tl.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, r in (d.items() if isinstance(d, dict) else enumerate(d)):
    print(k, json.dumps(r)[:1500])
PY
