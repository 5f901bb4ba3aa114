"""distributed_neural_networks_amd — MI355X-native pipeline-parallel inference engine.

Same capabilities as 123-code/Distributed-neural-networks (``node.py`` CLI,
``config.json`` partition schema, full-model ``.pth`` loading, gRPC
``NodeService``), re-designed for AMD Instinct MI355X (gfx950):

* ``models/``   golden torch models (CIFAR-10 ConvNet, GPT-2/nanoGPT, Llama-3)
* ``ops/``      hand-written HIP/CDNA4 kernels (MFMA GEMM, fused conv/pool,
                flash attention, norms, RoPE, fp8) behind thin Python wrappers
* ``parallel/`` partitioning, stage links (colocated / RCCL P2P / gloo / gRPC),
                pipeline schedules (GPipe fill-drain, decode ring)
* ``runtime/``  stage executors, HIP-graph capture, device engines
* ``wire/``, ``control/``  protobuf schema + gRPC control / CPU data plane
* ``utils/``    logging, metrics, tracing
"""
__version__ = "0.1.0"
