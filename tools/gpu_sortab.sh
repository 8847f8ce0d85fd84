# Sort gather A/B (TBC_SORT_GATHER_NT): kernel trace and FETCH_SIZE of the
# config 3 sort probe, default vs nontemporal gather loads -> gpurun_out/sortab/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sortab
mkdir -p $O
for v in base nt; do
  if [ $v = nt ]; then E="TBC_SORT_GATHER_NT=1"; else E="TBC_SORT_GATHER_BASE=1"; fi
  export $E
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$v -o run -- python3 -u tools/sort_probe.py --config 3 --reps 10 > $O/tr_$v.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python3 -u tools/sort_probe.py --config 3 --reps 3 > $O/fetch_$v.log 2>&1 || exit $?
  unset TBC_SORT_GATHER_NT TBC_SORT_GATHER_BASE
  grep '^{' $O/tr_$v.log
done
echo SORTAB_OK
