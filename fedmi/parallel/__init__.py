"""Data-plane parallelism: FedAvg collectives, compression, elastic groups."""
