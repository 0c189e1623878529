mkdir -p gpurun_out; : > gpurun_out/vbfb.txt
for vf in 16:8 8:4 4:2 2:1 1:1; do
  VB=${vf%%:*} FB=${vf##*:} QE="8:4" SH="8 2" bash tools/rt_fresh.sh || exit 1
  cat gpurun_out/rt_fresh.txt >> gpurun_out/vbfb.txt
done
