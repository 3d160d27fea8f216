"""Multi-GPU execution: tensor-parallel engine worker groups (one process per GPU, RCCL over
xGMI for the collectives, a gloo group for the leader's control broadcasts) and request-level
data parallelism (engine replicas behind the gateway / federated load balancer)."""
