"""CIFAR model zoo (reference src/models/*). Populated module by module."""
