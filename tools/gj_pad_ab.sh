set -o pipefail
for p in 0 24; do echo "pad $p KB"; SGP_GJ_PAD_KB=$p timeout -k 10 60 ./tools/micro/gj_trace | grep -v "^ *[0-9]* *[0-9]* *[0-9]* *[0-9]* *[0-9]*  next" || exit 1; done
