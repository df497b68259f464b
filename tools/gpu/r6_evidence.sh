# Round 6 evidence on the final sources: calibrations + PMC records (r6_pmcall.sh), then
# the final tests / smoke / bench / kernel stats / shard probe (r6_final.sh).
set -o pipefail
bash tools/gpu/r6_pmcall.sh && bash tools/gpu/r6_final.sh
