"""ddpx.optim."""
