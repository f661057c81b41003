#!/bin/bash
# pipelined forward as the default: the forward's HBM traffic, a bench line
O=gpurun_out
bash tools/pmc_attn_traffic.sh $O/r05x_pmc_traffic > $O/r05x_pmc.log 2>&1 || { tail -5 $O/r05x_pmc.log; exit 1; }
grep -h '"hbm_bytes_per_launch"\|"kernel"' $O/r05x_pmc_traffic/traffic_attn_fwd3_kernel.json
timeout -k 10 300 python -u bench.py --no-extras --cpu-baseline off > $O/r05x_bench.log 2>&1 || { tail -5 $O/r05x_bench.log; exit 1; }
grep '"metric"' $O/r05x_bench.log | cut -c1-300
