# Config 2 (DQN Pong) learner loop: the in-tree library vs alternate builds, alternating
#   bash tools/gpu_dqn_ab.sh ab/A/libdopamine_amd.so ...
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for lib in "" "$@"; do
    v=$(DOPAMINE_AMD_LIB=$lib timeout -k 10 240 python tools/dqn_chunk_ab.py 3 3000 2>&1 | tail -1) || exit 1
    echo "[${lib:-in-tree}] $v"
  done
done
