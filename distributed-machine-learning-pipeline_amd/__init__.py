"""hipdsml — MI355X-native distributed ML pipeline.

A brand-new, MI355X-first framework with the capabilities of
Helenbzbz/Distributed-Machine-Learning-Pipeline (a Go/gRPC simulator): the same
``gpu_sim`` gRPC control plane (coordinator + device servers, CommInit /
Memcpy / AllReduceRing / NaiveAllReduce / Group* / health monitor), but device
servers own real gfx950 GPUs, the MLP step runs as hand-written CDNA4 HIP
kernels (MFMA, LDS-resident row chain, fused SGD, hipGraph capture), and
gradient sync is a real ring all-reduce over RCCL send/recv on xGMI.

Import layout (the package directory is ``distributed-machine-learning-pipeline_amd``;
``hipdsml`` is its importable alias):

  hipdsml.models    MLP spec / layout / reference math
  hipdsml.ops       native loader + tensor ops (HIP on GPU, torch on CPU)
  hipdsml.engine    data-parallel trainer
  hipdsml.parallel  process groups, native RCCL comm, collectives
  hipdsml.runtime   device runtime (HBM arena, copy engine, stream table)
  hipdsml.rpc       gpu_sim gRPC API: coordinator, device server, client
  hipdsml.data      MNIST idx loader + synthetic data
  hipdsml.utils     config, metrics, tracing
"""
__version__ = "0.1.0"
