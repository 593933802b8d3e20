#!/bin/bash
# A/B of the contraction's grouped tile order (SGP_CON_GROUP) on C3: parity of the two orders
# at n=50000 m=1024, alternating bench runs, kernel statistics and FETCH_SIZE per order.
#   usage (inside gpurun): bash tools/gpu_r3_grp.sh
set -o pipefail
D=gpurun_out/grp
mkdir -p $D
export TMPDIR=/tmp
cat > /tmp/grp_par.py <<'PY'
import numpy as np, sparsergps_amd as S
from collections import OrderedDict
g = np.random.default_rng(3); n, m, d = 50000, 1024, 8
X = g.uniform(0, 10, (n, d)); U = g.uniform(0, 10, (m, d)); y = np.sin(X).sum(1) + g.normal(0, .3, n)
cp = OrderedDict(sigma=1.0, l=2.5, tau=0.5)
o, gr = S.vi_eval(cp, "sqexp", U, X, y, np.full(n, y.mean()), 1e-6)
print(repr(o), [repr(gr[k]) for k in cp])
PY
for v in 0 1; do SGP_CON_GROUP=$v PYTHONPATH=$PWD timeout -k 10 120 python3 /tmp/grp_par.py > $D/par$v.txt 2>&1 || exit 1; cat $D/par$v.txt; done
for r in 1 2 3; do for v in 0 1; do
  SGP_CON_GROUP=$v timeout -k 10 150 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $D/b$v.$r.json 2> $D/b$v.$r.err || exit 1
  echo "g=$v $(cut -c1-120 $D/b$v.$r.json)"
done; done
for v in 0 1; do
  SGP_CON_GROUP=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/k$v -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $D/k$v.json 2> $D/k$v.err || exit 1
  SGP_CON_GROUP=$v timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pf$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $D/pf$v.json 2> $D/pf$v.err || exit 1
done
echo done
