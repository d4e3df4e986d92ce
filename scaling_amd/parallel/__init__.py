"""Communication layer: TP/SP region collectives, DP gradient buckets, pipeline p2p (RCCL over xGMI)."""
