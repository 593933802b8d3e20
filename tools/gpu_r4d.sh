# C2 kernel traces: product library vs variants (SGP_AB_LIB), one short bench each
set -o pipefail
D=gpurun_out/r4d
mkdir -p $D
export TMPDIR=/tmp
for v in cur base notail; do
  if [ "$v" = cur ]; then unset SGP_AB_LIB; else export SGP_AB_LIB=tools/ab/$v/libsgp.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/$v -o run -- python3 bench.py --config C2 --steps 20 --warmup 3 --no-cpu-baseline > $D/$v.json 2> $D/$v.err || { tail -20 $D/$v.err; exit 1; }
done
ls $D/*
