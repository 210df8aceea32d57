"""Runtime: flat parameter store, fused trainer, checkpointing, optimizer state."""
