# Submit one gpurun call, resubmitting ONLY while gpurun answers 3 ("no box
# or slot free right now": nothing ran, nothing was charged).  Any other exit
# status -- success, a failed command, a timeout -- ends the loop: a GPU step
# that ran is never repeated.
#   bash tools/gpurun_queue.sh OUTFILE TIMEOUT_S 'command'
out=$1
lim=$2
cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  transient=0
  [ $rc -eq 3 ] && transient=1
  grep -q "status=transient" "$out" && grep -q "nothing was charged" "$out" && transient=1
  if [ $transient -eq 0 ]; then
    echo "gpurun rc=$rc (attempt $i)" >> "$out"
    exit $rc
  fi
  sleep 90
done
echo "gave up after 40 attempts" >> "$out"
exit 3
