set -o pipefail
mkdir -p gpurun_out/bt
( cd tools/micro && for b in con_trace_base ct_v1 ct_v2 ct_base_lone ct_v1_lone ct_v2_lone con_trace_base ct_v1 ct_v2; do echo "== $b"; timeout -k 10 60 ./$b /tmp/x.csv | grep "^run 2" || exit 1; done ) || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > gpurun_out/bt/pytest.log 2>&1; tail -3 gpurun_out/bt/pytest.log
for rep in 1 2; do for v in cur prev; do
  cp sparsergps_amd/lib/libsgp_$v.so sparsergps_amd/lib/libsgp.so
  timeout -k 10 300 python3 bench.py --mode fitc --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bt/fitc_$v$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bt/c3_$v$rep.json 2>/dev/null || exit 1
  python3 -c "
import json
for f in ['fitc','c3']:
  d=json.load(open('gpurun_out/bt/'+f+'_$v$rep.json')); p=d['phases_ms']
  print('$v $rep', f, round(d['value'],3), {k:round(v,2) for k,v in p.items() if v>1})"
done; done
cp sparsergps_amd/lib/libsgp_cur.so sparsergps_amd/lib/libsgp.so
