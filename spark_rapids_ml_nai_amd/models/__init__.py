"""Spark-free device solvers: each takes rank-local device tensors + a WorkerContext."""
