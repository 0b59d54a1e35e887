#!/usr/bin/env bash
# Build (and optionally push) the origin (ROCm + engine) and edge (native server only) images.
#   scripts/build-images.sh [registry] [tag] [--push]
set -euo pipefail
cd "$(dirname "$0")/.."
REG=${1:-registry.example.com/dsse}
TAG=${2:-latest}
docker build -f deploy/docker/Dockerfile -t "$REG/origin:$TAG" .
docker build -f deploy/docker/Dockerfile.edge -t "$REG/edge:$TAG" .
if [[ "${3:-}" == "--push" ]]; then
  docker push "$REG/origin:$TAG"
  docker push "$REG/edge:$TAG"
fi
