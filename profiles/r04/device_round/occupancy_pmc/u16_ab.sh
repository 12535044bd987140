set -uo pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/u16_ab
mkdir -p $O
L=mobile-federated-learning_amd/lib/libfedavg_amd.so
for V in base u16 base2 u16b base3 u16c; do
  S=${V%[23]}; S=${S%[bc]}
  cp jobs/lib_$S.so $L
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$V -o run -- python scripts/segwin_layout_probe.py --config resnet56 --calls 30 --layout separate > $O/$V.log 2>&1 || exit 1
  find $O/$V -name '*trace*.csv' -delete
  echo $V done
done
cp jobs/lib_u16.so $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_device_round.py tests/test_gpu_model_shapes.py tests/test_gpu_device_clients.py tests/test_gpu_window.py > $O/test_u16.log 2>&1 || { tail -20 $O/test_u16.log; exit 1; }
echo test_u16 $(tail -1 $O/test_u16.log)
