# drop-in NaN: which host synchronisation point removes it (noautograd loop)
for at in next col fwd bwd opt; do
  SYNC_AT=$at timeout -k 10 200 python3 tools/dropin_debug3.py noautograd > gpurun_out/sync_$at.log 2>&1 || exit 1
  echo "sync at $at: $(grep -h 'losses' gpurun_out/sync_$at.log)"
done
