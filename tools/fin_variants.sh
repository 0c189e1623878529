# k_finish vertex layout (PSGPU_OPT_FINISH_QUAD 0: one lane per vertex, 1: a quad of lanes per
# vertex, 2: chosen per run) at strong-scaling rank shares, alternating on one box:
# tools/range_test.py with FQ=<mode>, FB=<persistent blocks per CU>.  Results in gpurun_out/fin.txt.
mkdir -p gpurun_out; o=gpurun_out/fin.txt; : > $o
for r in 1 2; do for fq in ${MODES:-0 1 2}; do for fb in ${FBS:-8 4}; do
  GPU_MAX_HW_QUEUES=8 ENGINES=4 SHARES=${SHARES:-8,4} FQ=$fq FB=$fb timeout -k 10 120 python3 -u tools/range_test.py >> $o 2>&1 || exit 1
done; done; done
