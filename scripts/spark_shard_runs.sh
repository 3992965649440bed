set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload spark --log-nnz 24 --steps 3 --warmup 1 > gpurun_out/spark24_n1.json 2> gpurun_out/spark24_n1.err || exit $?
echo n1 done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload spark --backend gloo --log-nnz 24 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/spark24_n4.json 2> gpurun_out/spark24_n4.err || exit $?
echo n4 done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --workload spark --backend gloo --log-nnz 20 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/spark20_n2.json 2> gpurun_out/spark20_n2.err || exit $?
echo n2 done
