"""ddpx.data."""
