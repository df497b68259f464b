# Round 6 combined step: the GPU suite, init-regime A/B of $CFGS (this build vs
# HEAD-of-round), config 3's first sweep profile, config 2's write attribution.
set -o pipefail
export PYTHONUNBUFFERED=1
TAG=${TAG:-r6combo} CFGS=${CFGS:-cfg2,cfg5} LIBS=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base6.so REPS=${REPS:-3} bash tools/gpu/r6.sh || exit $?
TAG=${TAG:-r6combo}_first bash tools/gpu/r6_first.sh || exit $?
TAG=${TAG:-r6combo}_writes bash tools/gpu/r6_writes.sh || exit $?
