set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/occ_ab
mkdir -p $O
L=mobile-federated-learning_amd/lib/libfedavg_amd.so
cp $L jobs/lib_base.so
for V in base w5 w6 base2 w5b w6b; do
  S=${V%2}; S=${S%b}
  cp jobs/lib_$S.so $L
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$V -o run -- python scripts/segwin_layout_probe.py --config resnet56 --calls 30 --layout separate > $O/$V.log 2>&1 || exit 1
  grep -h "segments_f32_kernel<64, true>" $O/$V/run_kernel_stats.csv | cut -d, -f2-8 > $O/$V.stat
  echo $V $(cat $O/$V.stat) $(tail -c 400 $O/$V.log | grep -o '"round_gpu_us_median": [0-9.]*')
  find $O/$V -name '*trace*.csv' -delete
done
for V in w5 w6; do
  cp jobs/lib_$V.so $L
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_device_round.py tests/test_gpu_model_shapes.py > $O/test_$V.log 2>&1 || { tail -20 $O/test_$V.log; exit 1; }
  echo test_$V $(tail -1 $O/test_$V.log)
done
cp jobs/lib_base.so $L
