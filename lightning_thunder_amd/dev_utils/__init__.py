"""Developer utilities: trace checking, profiling transforms, debug transforms."""
