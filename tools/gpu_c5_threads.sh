cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out
for r in 1 2; do for h in 1 2; do
timeout -k 10 200 python -u tools/c5_run.py --steps 12 --no-parity --host-threads $h > $O/c5ht_$h.log 2>&1 || exit $?
echo "threads $h $(tail -1 $O/c5ht_$h.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["ms_per_step_serial"])')"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c5ht_prof -o run --output-format csv -- python3 tools/c5_run.py --no-parity --steps 6 --host-threads 2 > $O/c5ht_prof.log 2>&1 || exit $?
python3 tools/timeline.py $O/c5ht_prof --min-us 20 > $O/c5ht_timeline.txt 2>&1 || true
