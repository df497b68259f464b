#!/usr/bin/env bash
# round 4 session 3: EK=4 sweep kernel — parity subset, A/B against the HEAD build,
# then the fine per-sequence timeline (TLF marks) of config 2 init
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${PYT:-tests/test_gpu_parity.py tests/test_gpu_fullsize_sweep.py tests/test_golden.py tests/test_gpu_dna.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/ab.sh s4ab cfg2,cfg5 init gibbssampling_amd/libgibbs_hip_base.so,gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base.so,gibbssampling_amd/libgibbs_hip.so 100 || exit 1
GS_TL_LIB=libgibbs_hip_tlf.so timeout -k 10 240 python tools/timeline.py cfg2:init > $O/timeline_fine.json 2> $O/timeline.err || { tail -20 $O/timeline.err; exit 1; }
python - <<'P'
import json
d=json.load(open('gpurun_out/s4/timeline_fine.json'))
for k,v in d.items():
    for r in v['runs']:
        print(k, {x:r[x] for x in r if x.startswith("m") or x in ("wave_life_us",)})
P
