timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t6.log 2>&1; tail -3 gpurun_out/t6.log
bash tools/ab_libs.sh "graph_neural_cellular_automata_amd/libgnca.so build_ab/lib_noimg.so build_ab/lib_prio0.so build_ab/lib_nosub.so" headline 2
bash tools/ab_libs.sh "graph_neural_cellular_automata_amd/libgnca.so build_ab/lib_noimg.so" c3 2
bash tools/ab_libs.sh "graph_neural_cellular_automata_amd/libgnca.so build_ab/lib_noimg.so" c2 1
