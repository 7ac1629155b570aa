#!/bin/bash
# Container entry point (parity: reference build_files/start.sh:88-126).
#   MODEL_CACHE=tmpfs  copy $MODEL_SRC into /dev/shm (fast cold start; 288 GB HBM holds the stacks)
#   MODEL_CACHE=nfs    use $MODEL_SRC in place through an extra_model_paths.yaml
#   GPUS=N             GPUs to serve (default: all visible)
#   SERVE=node         (default) ONE API for the whole node: `main.py --gpus $GPUS` -- rank 0 serves HTTP/WS
#                      on 8188 and coordinates, a prompt's image batch is split over all GPUs, independent
#                      prompts run concurrently on idle GPUs (sched/cluster.py)
#   SERVE=per-gpu      one independent server per GPU on 8188+i, nginx spreads clients (sticky per IP)
#   LATENCY=1          (node mode) batch-1 prompts split CFG / token parallel over the GPUs
#   GRPC=1             also serve comfy_request.v1 over gRPC (50051, or 50051+i per GPU)
set -euo pipefail
cd /gen-server
MODEL_SRC=${MODEL_SRC:-/runpod-volume/models}
MODEL_CACHE=${MODEL_CACHE:-nfs}
if [ -z "${GPUS:-}" ]; then GPUS=$(python -c "import torch; print(max(1, torch.cuda.device_count()))"); fi

if [ -d "$MODEL_SRC" ]; then
  if [ "$MODEL_CACHE" = "tmpfs" ]; then
    mkdir -p /dev/shm/models && cp -rn "$MODEL_SRC"/. /dev/shm/models/
    ROOT=/dev/shm/models
  else
    ROOT=$MODEL_SRC
  fi
  cat > /gen-server/extra_model_paths.yaml <<YAML
shared:
  base_path: $ROOT
  checkpoints: checkpoints
  vae: vae
  loras: loras
  controlnet: controlnet
  clip: clip
  clip_vision: clip_vision
  upscale_models: upscale_models
  embeddings: embeddings
  unet: unet
YAML
  EXTRA="--extra-model-paths-config /gen-server/extra_model_paths.yaml"
else
  EXTRA=""
fi

upstreams=""
if [ "${SERVE:-node}" = "node" ]; then
  grpc=""
  if [ "${GRPC:-0}" = "1" ]; then grpc="--grpc-port 50051"; fi
  lat=""
  if [ "${LATENCY:-0}" = "1" ]; then lat="--latency-mode"; fi
  MASTER_ADDR=127.0.0.1 python main.py --listen 0.0.0.0 --port 8188 --gpus "$GPUS" --disable-metadata $EXTRA $grpc $lat &
  upstreams="    server 127.0.0.1:8188;\n"
else
  for ((i = 0; i < GPUS; i++)); do
    port=$((8188 + i))
    grpc=""
    if [ "${GRPC:-0}" = "1" ]; then grpc="--grpc-port $((50051 + i))"; fi
    HIP_VISIBLE_DEVICES=$i python main.py --listen 0.0.0.0 --port "$port" --disable-metadata $EXTRA $grpc &
    upstreams="$upstreams    server 127.0.0.1:$port;\n"
  done
fi
sed -i "s|# UPSTREAMS|$upstreams|" /etc/nginx/nginx.conf
nginx
wait -n
