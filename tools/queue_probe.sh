mkdir -p gpurun_out; o=gpurun_out/qp.txt; : > $o
export GPU_MAX_HW_QUEUES=${Q:-8}
for v in ${VARIANTS:-"0:0:0 1:0:0"}; do
  IFS=: read x p t vb fb <<< "$v"
  EXTRA=$x PRERUN=$p TORCH=$t VB=${vb:-0} FB=${fb:-0} timeout -k 10 60 python -u tools/queue_probe.py >> $o 2>&1 || exit 1
done
