# Runs one gpurun call in the background of this container, retrying only while the pool reports a
# transient infrastructure status (no box, box lost before the command ran: nothing charged); the
# command itself is never re-run after it has started.  usage: bash tools/gpurun_bg.sh LOG TIMEOUT 'CMD'
LOG=$1; TO=$2; CMD=$3
echo $$ > $LOG.pid   # this loop's own PID, to stop it by that number
for k in $(seq 1 12); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient rc=None" $LOG; then sleep 150; continue; fi
  if [ $rc = 3 ]; then sleep 180; continue; fi   # no box or slot free right now (nothing charged)
  exit $rc
done
