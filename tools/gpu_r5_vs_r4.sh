# round 5 against round 4 on one box: HEAD ("cur") alternating with the round-4 head's library (r4,
# commit c900cc1), every bench line of the round's closing run
set -o pipefail
bash tools/ab.sh v4c2 4 "r4" --config C2 --steps 300 --warmup 20 || exit 1
bash tools/ab.sh v4c3 3 "r4" --steps 10 --warmup 2 || exit 1
bash tools/ab.sh v4fitc 2 "r4" --mode fitc --steps 6 --warmup 2 || exit 1
bash tools/ab.sh v4c5 2 "r4" --config C5 --mode laplace --steps 10 --warmup 2 || exit 1
bash tools/ab.sh v4sh 2 "r4" --n 125000 --steps 40 --warmup 4 || exit 1
