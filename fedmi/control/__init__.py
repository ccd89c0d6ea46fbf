"""gRPC control plane (federated.Trainer service)."""
