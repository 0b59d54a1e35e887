#!/usr/bin/env bash
# Deploy one region.
#   scripts/deploy.sh origin <kubeconfig>                 # GPU origin (8x MI355X node) + monitoring
#   scripts/deploy.sh edge   <kubeconfig> <origin-host>   # delivery-only edge relaying from the origin
# Waits for the rollout and prints the public endpoints (compare reference scripts/deploy-origin.sh and
# scripts/deploy-edge.sh; no NATS leaf credentials or IP sed-substitution into base manifests here:
# the origin address is a kustomize patch rendered into a temp overlay).
set -euo pipefail
cd "$(dirname "$0")/.."
ROLE=${1:?origin|edge}
export KUBECONFIG=${2:?kubeconfig}
K="kubectl"
case "$ROLE" in
  origin)
    $K apply -k deploy/kubernetes/overlays/origin
    $K -n dsse rollout status deploy/dsse-origin --timeout=1800s
    ;;
  edge)
    ORIGIN=${3:?origin public host}
    TMP=$(mktemp -d)
    cp -r deploy/kubernetes/overlays/edge/. "$TMP/"
    sed -i "s#ORIGIN_HOST#${ORIGIN}#g" "$TMP/origin-address.yaml"
    sed -i "s#\.\./\.\./base#$(pwd)/deploy/kubernetes/base#g" "$TMP/kustomization.yaml"
    $K apply -k "$TMP"
    rm -rf "$TMP"
    $K -n dsse rollout status deploy/dsse-edge --timeout=600s
    ;;
  *) echo "unknown role $ROLE" >&2; exit 2 ;;
esac
$K -n dsse get svc -o wide
