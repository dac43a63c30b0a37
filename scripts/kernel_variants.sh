# Per-kernel A/B of the variant libraries in build/var: one rocprofv3 kernel trace per variant,
# prints the average duration of every kernel whose name matches $1.
#   bash scripts/kernel_variants.sh <name-regex> <command args...>
set -u
export TMPDIR=/tmp
pat=$1; shift
OUT=gpurun_out/kvar; mkdir -p $OUT
for r in 1 2; do for so in build/var/libdadmm_*.so; do
  v=$(basename $so .so)
  DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v.$r -o run -- "$@" > $OUT/$v.$r.log 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; exit $rc; fi
  f=$(find $OUT/$v.$r -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$pat" "$v" <<'PY'
import csv, re, sys
for row in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], row["Name"]):
        print(f"{sys.argv[3]:24s} {float(row['AverageNs']) / 1e3:9.1f} us x{row['Calls']:>4}  {row['Name'][:70]}")
PY
done; done
