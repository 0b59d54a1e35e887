# Multi-region layout: one GPU origin and any number of delivery-only edges (the reference's
# terraform/main.tf regions map: us-ord origin, us-lax / us-mia edges).
variable "origin_kubeconfig" { type = string }
variable "origin_public_host" {
  type        = string
  description = "LoadBalancer address of service dsse/dsse-origin-public"
}
variable "edge_kubeconfigs" {
  type    = map(string)
  default = {}
  description = "region name -> kubeconfig path"
}

module "origin" {
  source     = "./modules/dsse-region"
  role       = "origin"
  kubeconfig = var.origin_kubeconfig
  repo_root  = abspath("${path.root}/../..")
}

module "edge" {
  for_each    = var.edge_kubeconfigs
  source      = "./modules/dsse-region"
  role        = "edge"
  kubeconfig  = each.value
  origin_host = var.origin_public_host
  repo_root   = abspath("${path.root}/../..")
  depends_on  = [module.origin]
}
