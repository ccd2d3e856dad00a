"""ddpx.train."""
