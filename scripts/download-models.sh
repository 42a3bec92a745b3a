#!/usr/bin/env bash
# Fetch the GGUF checkpoints named in config/default-config.toml into $AIOS_MODEL_DIR
# (needs network access; the benchmarks and tests never call this -- they use random-init
# weights of the same architectures).
#   scripts/download-models.sh [--tactical] [--strategic]
set -euo pipefail
DIR=${AIOS_MODEL_DIR:-/var/lib/aios/models}; mkdir -p "$DIR"
fetch() {  # url file min_bytes
  local out="$DIR/$2"
  if [ -f "$out" ] && [ "$(stat -c %s "$out")" -ge "$3" ]; then echo "have $2"; return; fi
  curl -fL --retry 3 -o "$out.part" "$1" && mv "$out.part" "$out"
  [ "$(stat -c %s "$out")" -ge "$3" ] || { echo "$2 too small"; rm -f "$out"; exit 1; }
}
fetch https://huggingface.co/TheBloke/TinyLlama-1.1B-Chat-v1.0-GGUF/resolve/main/tinyllama-1.1b-chat-v1.0.Q4_K_M.gguf \
  tinyllama-1.1b-chat-v1.0.Q4_K_M.gguf 600000000
for a in "$@"; do
  case "$a" in
    --tactical) fetch https://huggingface.co/TheBloke/Mistral-7B-Instruct-v0.2-GGUF/resolve/main/mistral-7b-instruct-v0.2.Q4_K_M.gguf \
      mistral-7b-instruct-v0.2.Q4_K_M.gguf 4000000000 ;;
    --strategic) echo "place a Llama-3-70B-Instruct Q4_K_M GGUF at $DIR/llama-3-70b-instruct.Q4_K_M.gguf (gated download)" ;;
  esac
done
