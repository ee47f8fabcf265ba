# round-3 final measurement, part 2: rocprof stats + PMC traffic of configs[2] train / configs[1]
# infer and of YOLO-MS-S training, plus the traced-step timeline
set -e
TAG=${1:-r03b}
bash tools/profile_round.sh $TAG
MODES=train EXTRA="--version ms-s" bash tools/profile_round.sh ${TAG}_ms_s
echo "profiles done"
