"""ddpx.ops."""
