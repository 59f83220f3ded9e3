set -e
for L in distilp_amd/libhalda.so build/variants/libhalda_nopf4.so build/variants/libhalda_nopf6.so; do
  HALDA_LIB=$L timeout -k 10 200 python -u tools/ab_c3.py >> gpurun_out/r5_ab1.log 2>&1
done
