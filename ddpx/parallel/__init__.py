"""ddpx.parallel."""
