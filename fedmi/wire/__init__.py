"""Wire layer: federated.proto messages/stubs and the checkpoint codec."""
