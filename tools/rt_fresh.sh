# strong-scaling rehearsal sweep: each (hw queues, engines, rank share) in a fresh process
mkdir -p gpurun_out
out=gpurun_out/rt_fresh.txt; : > $out
for qe in ${QE:-"4:2 8:4"}; do q=${qe%%:*}; e=${qe##*:}; for s in ${SH:-1 8}; do
  echo "q=$q" >> $out
  GPU_MAX_HW_QUEUES=$q ENGINES=$e SHARES=$s VB=$VB FB=$FB timeout -k 10 60 python -u tools/range_test.py >> $out 2>&1 || exit 1
done; done
