"""tony_amd: an MI355X-native distributed deep-learning job launcher with TonY's
capabilities (tony.xml schema, ClusterSubmitter CLI, TF/PyTorch/MXNet/Horovod
runtimes) plus the training hot path of its reference jobs as CDNA4 HIP kernels
and RCCL-over-xGMI collectives.  See SURVEY.md for the component map.
"""
__version__ = "0.1.0"
