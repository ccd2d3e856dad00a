"""ddpx.utils."""
