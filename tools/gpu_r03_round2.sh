# round-3 mid snapshot, part 2: rocprof stats + PMC traffic of configs[2]/[1] and of YOLO-MS-S train
set -e
TAG=${1:-r03a}
bash tools/profile_round.sh $TAG
MODES=train EXTRA="--version ms-s" bash tools/profile_round.sh ${TAG}_ms_s
