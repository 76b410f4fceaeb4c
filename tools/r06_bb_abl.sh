# round 6: BB timing variants at B=1024 72^2 (tools/time_bwd.py), interleaved with the product library
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do for lib in graph_neural_cellular_automata_amd/libgnca.so ${ABL_LIBS:-build_ab/lib_abl_store.so}; do
  echo "== $lib"; GNCA_LIB_PATH=$lib timeout -k 10 200 python tools/time_bwd.py --sizes ${ABL_SIZES:-1024x72} --iters 10 2>&1 | grep "B=" || exit 1
done; done
