bash tools/ab_libs.sh "graph_neural_cellular_automata_amd/libgnca.so build_ab/lib_prio2.so build_ab/lib_prio3.so build_ab/lib_nosub.so" headline 2
echo "=== ablation headline"
ABLATE_ONLY=full,lds_linear,no_gather,no_perceive,no_mfma,mfma_only,prof ABLATE_PROF_SETS=w03 timeout -k 10 300 python tools/ablate.py run 2>&1 | grep -v amdgpu.ids
echo "=== ablation c3"
ABLATE_CONFIG=c3 ABLATE_ONLY=full,no_tiles,no_tiles_no_fill,prof ABLATE_PROF_SETS=w03 ABLATE_PHASES=2 timeout -k 10 300 python tools/ablate.py run 2>&1 | grep -v amdgpu.ids
