"""Shared parameters: CPU-runtime KV objects and the GPU sharded KV store."""
