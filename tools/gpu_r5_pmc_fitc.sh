# round 5: HBM traffic of FITC's one-pass stored-product gradient contraction (k_contract T2):
# separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH HBM section)
set -o pipefail
D=gpurun_out/pmcfitc
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python3 bench.py --no-cpu-baseline --mode fitc --steps 2 --warmup 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pf -o run -- $B > $D/pf.json 2> $D/pf.err || { tail -20 $D/pf.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/pw -o run -- $B > $D/pw.json 2> $D/pw.err || { tail -20 $D/pw.err; exit 1; }
F=$(ls $D/pf/*counter_collection.csv | head -1); W=$(ls $D/pw/*counter_collection.csv | head -1)
python3 tools/pmc_traffic.py $F $W --n 1000000 --m 1024 --match "k_contract<8, 0, false, false, true, true, true>" --out $D/traffic_t2.json
python3 tools/pmc_traffic.py $F $W --n 1000000 --m 1024 --match "k_contract<8, 1, false, false, false, true, false>" --out $D/traffic_rowquad_p.json || true
