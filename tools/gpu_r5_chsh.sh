# round 5: FITC / C5 builder share beside the (persistent) K22 chain -- chain_shared_rb's model
set -o pipefail
bash tools/ab.sh chf 2 "ch25 ch40 ch0" --mode fitc --steps 6 --warmup 2 || exit 1
bash tools/ab.sh chl 2 "ch25 ch40 ch0" --config C5 --mode laplace --steps 10 --warmup 2 || exit 1
