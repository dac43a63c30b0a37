# End-to-end A/B of the variant libraries in build/var on the GNN model forward (eval, no_grad):
# configs[4]'s per-GPU shard (P=50, n=1024, K=5) and the P=5 headline-size model (K=25).
set -u
for r in 1 2; do for so in build/var/libdadmm_*.so; do
  for shape in "1024 50 1024 32 5 3" "1024 5 256 64 25 3"; do
    DADMM_LIB_VARIANT=$PWD/$so timeout -k 10 200 python3 scripts/prof_gnn.py $shape | sed "s|^|$(basename $so) |"
    rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done; done
