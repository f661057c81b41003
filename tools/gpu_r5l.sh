# NT / TN token GEMMs vs hipBLASLt under a kernel trace: which library kernels (tile configs in their names) win
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/r5l; mkdir -p $O
timeout -k 10 200 python3 tools/gemm_vs_blas.py 5 > $O/gemm_vs_blas.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 tools/gemm_vs_blas.py 2 > $O/traced.log 2>&1 || exit 4
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv; rm -rf $O/p
