# one gpu_profile.sh group per call (the call limit): bash tools/r03_prof.sh <tag> <group>
set -o pipefail
GROUPS_TO_RUN="$2" bash "$GRAFT_REPO_ROOT/tools/gpu_profile.sh" "$1"
