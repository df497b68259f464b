#!/usr/bin/env bash
# round 4 session 3: live kernel with kernarg reads at use — its parity tests, config
# 3/4 init A/B against the round-start build, the init-regime shard table
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dna.py tests/test_gpu_long.py tests/test_gpu_fullsize_sweep.py tests/test_gpu_bg.py tests/test_gpu_dist_gloo.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/ab.sh s6ab cfg4,cfg3 init gibbssampling_amd/libgibbs_hip_base.so,gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base.so,gibbssampling_amd/libgibbs_hip.so 30 || exit 1
timeout -k 10 400 python tools/shard_probe.py --config cfg4 --worlds 1,2,4,8 --steps 6 --tunings ";live_G=1,live_waves=4" > $O/shard.jsonl 2> $O/shard.err || { tail -20 $O/shard.err; exit 1; }
python -c "
import json
for l in open('$O/shard.jsonl'):
    d=json.loads(l); print(d['world'], d['tuning'], round(d['us_per_sweep_kernel'],1), d['positions_match_whole_sampler'], d['keep_motif'])
"
