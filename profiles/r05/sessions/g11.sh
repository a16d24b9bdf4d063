set -o pipefail
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/g11; mkdir -p $O
for v in 1024 128; do
  timeout -k 10 300 python tools/first_step.py --videos $v --steps 20 --warmup 5 2>&1 | grep -v amdgpu.ids | tee $O/first_v$v.log || exit $?
  timeout -k 10 300 python tools/first_step.py --videos $v --steps 20 --warmup 5 --spin 50 2>&1 | grep -v amdgpu.ids | tee $O/first_spin_v$v.log || exit $?
done
