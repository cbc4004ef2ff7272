"""Developer utilities: trace checking, debug/profile transforms, roctx ranges, benchmarking
(reference ``thunder/dev_utils``)."""
