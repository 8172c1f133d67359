set -e
mkdir -p gpurun_out
python tools/mk_synth.py 600 /tmp/a.npy
for K in 1 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node $K --master-addr 127.0.0.1 --master-port 29611 tools/dist_transcribe.py /tmp/a.npy --model large-v3 --seg vad --backend gloo --device 0 --strategy greedy --force-len 3.3 --spurts /tmp/a.npy.json --out gpurun_out/k$K.json 2> gpurun_out/k$K.err
  grep "rank" gpurun_out/k$K.err
done
