# Round 6 combined step 3: the GPU suite; init-regime A/B of configs 2, 3, 5 against
# HEAD-of-round; config 3's first sweep from uniform starts (profiled); the write and
# fetch counters of configs 2 and 5.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${TAG:-r6c3}
TAG=$T CFGS=cfg2,cfg3,cfg4,cfg5 LIBS=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base6.so REPS=2 bash tools/gpu/r6.sh || exit $?
TAG=${T}_first bash tools/gpu/r6_first.sh || exit $?
TAG=${T}_wr bash tools/gpu/r6_wr.sh cfg2 cfg5 || exit $?
