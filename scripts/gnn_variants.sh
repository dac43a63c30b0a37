set -u
for r in 1 2; do for so in build/var/libdadmm_*.so; do
  DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 200 python3 scripts/prof_gnn.py 1024 50 1024 32 5 3 | sed "s|^|$(basename $so) |" ; rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
done; done
