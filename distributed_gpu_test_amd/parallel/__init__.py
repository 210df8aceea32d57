"""Data-parallel communication: process groups, bucketed RCCL collectives, IPC one-shot exchange."""
