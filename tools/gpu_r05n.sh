#!/bin/bash
# round-4 attention PMC retake: instruction / wait / LDS counters per pass (tools/pmc_attn.sh),
# the table, and HBM traffic per launch (tools/pmc_attn_traffic.sh)
#   gpurun --timeout 900 -- 'bash tools/gpu_r05n.sh'
O=gpurun_out
bash tools/pmc_attn.sh $O/r05n_pmc_attn || exit $?
for d in $O/r05n_pmc_attn/p*/; do f=$(find $d -name run_counter_collection.csv | head -1); [ -n "$f" ] && cp "$f" $d; done
python tools/pmc_table.py $O/r05n_pmc_attn/p1 $O/r05n_pmc_attn/p2 $O/r05n_pmc_attn/p3 $O/r05n_pmc_attn/p4 $O/r05n_pmc_attn/p5 > $O/r05n_pmc_attention_table.txt || exit $?
bash tools/pmc_attn_traffic.sh $O/r05n_pmc_traffic || exit $?
