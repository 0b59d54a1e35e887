# Deploys one region (origin or edge) of the stack onto an existing Kubernetes cluster by rendering the
# kustomize overlay and applying it with kubectl.  Cluster provisioning itself (the reference creates
# Linode LKE clusters with an RTX 4000 node pool, terraform/modules/lke-cluster) is cloud-specific: point
# `kubeconfig` at any cluster whose origin node pool carries 8x MI355X with the AMD GPU device plugin.
terraform {
  required_providers {
    null = { source = "hashicorp/null", version = ">= 3.2" }
  }
}

variable "role" {
  type        = string
  description = "origin | edge"
  validation {
    condition     = contains(["origin", "edge"], var.role)
    error_message = "role must be origin or edge"
  }
}
variable "kubeconfig" { type = string }
variable "repo_root" { type = string }
variable "origin_host" {
  type        = string
  default     = ""
  description = "public address of the origin (edges only)"
}

resource "null_resource" "deploy" {
  triggers = {
    role        = var.role
    kubeconfig  = var.kubeconfig
    origin_host = var.origin_host
    manifests   = sha1(join("", [for f in fileset("${var.repo_root}/deploy/kubernetes", "**") : filesha1("${var.repo_root}/deploy/kubernetes/${f}")]))
  }
  provisioner "local-exec" {
    command = var.role == "origin" ? "${var.repo_root}/scripts/deploy.sh origin ${var.kubeconfig}" : "${var.repo_root}/scripts/deploy.sh edge ${var.kubeconfig} ${var.origin_host}"
  }
}

output "role" { value = var.role }
