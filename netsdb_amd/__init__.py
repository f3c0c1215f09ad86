"""netsdb_amd — an MI355X-native UDF-centric analytics database with netsDB's capabilities.

Layers (see SURVEY.md / docs/ARCHITECTURE.md):
  objects/        PDB object model (typed records, columnar RecordBatch pages)
  lambdas/        UDF lambda trees (makeLambda, makeLambdaFromMember/Method/Self, ==, &&, ...)
  computations/   Selection / MultiSelection / Join / Aggregate / Partition / TopK / Scan / Write
  logical_plan/   TCAP compiler (+ native C++ TCAP parser in csrc/runtime)
  query_planning/ stage planner (pipelines, join strategy), tensor-pattern fusion onto MFMA kernels
  execution/      vectorised pipeline engine (GPU tensor columns), hash join / group-by primitives
  storage/        sets, pages, HBM budget + native buffer manager / page files, sqlite catalog
  parallel/       one process per GPU, RCCL collectives for shuffles/broadcasts, dispatcher policies
  ops/            CDNA4 HIP kernels (MFMA block GEMM, fused conv2d, softmax, LSTM cell, embeddings)
  la/             linear-algebra DSL (lexer/parser/evaluator over MatrixBlock sets)
  models/         FF-NN, conv2d (memory fusion + projection), LSTM, LogReg, word2vec, text classifier
  selflearning/   Lachesis-style partitioning advisor (rule-based + learned)
  server/         socket front end (master) for remote clients
"""
__version__ = "0.1.0"

from .objects import PDBObject, RecordBatch, Tensor, Vector  # noqa: F401


def __getattr__(name):
    if name == "PDBClient":
        from .client import PDBClient

        return PDBClient
    raise AttributeError(name)
