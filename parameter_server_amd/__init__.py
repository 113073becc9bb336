"""parameter_server_amd — an MI355X-native parameter server.

Colocated worker + HBM server shard per GPU, RCCL all-to-all over xGMI for
push/pull, hand-written HIP kernels (gfx950) for the sparse hot paths, and a
C++ host runtime (TCP van, config parser, data parsers) for the
scheduler/server/worker control plane.
"""
__version__ = "0.1.0"
