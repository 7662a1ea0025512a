"""distributed_machine_learning_amd — an MI355X-native distributed image-classification
inference service (capabilities of shahzadjutt123/Distributed-Machine-Learning,
re-designed for gfx950: hand-written MFMA HIP kernels, one process per GPU, RCCL
data plane over xGMI, host-side SWIM membership / election / fair-share scheduler).

Subpackages
  models    layer IR, ResNet50 / InceptionV3 graphs, fp32 oracle, native engine
  ops       functional wrappers of the gfx950 kernels
  parallel  RCCL data plane, pinned staging, per-GPU serving pipeline
  cluster   control plane: frames, transport, SWIM membership, election, introducer
  serving   jobs/batching, fair-share scheduler, coordinator, standby, metrics, CLI
  store     replicated versioned image store (SDFS equivalent)
  utils     config, logging, tracing, labels
"""
__version__ = "0.1.0"
