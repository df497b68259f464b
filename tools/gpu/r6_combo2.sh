# Round 6 combined step 2: the GPU suite, config 3 init A/B and first sweep from uniform
# starts (profiled), config 2's write attribution.
set -o pipefail
export PYTHONUNBUFFERED=1
T=${TAG:-r6c2}
TAG=$T CFGS=cfg3 LIBS=gibbssampling_amd/libgibbs_hip.so,gibbssampling_amd/libgibbs_hip_base6.so REPS=2 bash tools/gpu/r6.sh || exit $?
TAG=${T}_first bash tools/gpu/r6_first.sh || exit $?
TAG=${T}_writes bash tools/gpu/r6_writes.sh || exit $?
