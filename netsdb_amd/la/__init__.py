"""linearAlgebraDSL — a small matrix language compiled onto netsDB computations.

Reference: src/linearAlgebraDSL (LALexer.l, LAParser.y, LA*Node.h, LAEvaluateFunctions.cc,
LAPDBInstance.h; samples in DSLSamples/*.pdml; tests src/tests/source/TestLA*.cc).

    X = load(100,10,10,1,"X.data")        # blockRowSize, blockColSize, blockRowNum, blockColNum, file
    A = ones(20,20,10,10)   B = zeros(...)   I = identity(blockSize, blockNum)
    C = A %*% B   D = A '* B (=A^T B)   E = A * B (elementwise)   F = A + B   G = A - B
    H = A^T   J = A^-1   k = max(A)   min(A)   rowMax/rowMin/rowSum/colMax/colMin/colSum(A)
    duplicateRow(v, blockRowSize, blockRowNum)   duplicateCol(v, blockColSize, blockColNum)

Every operator becomes the corresponding LA UDF computation(s) (la/computations.py) executed
through PDBClient.execute_computations, so multiplies land on the split-K MFMA GEMM and, when
matrices are row-partitioned over GPUs, on the RCCL ring matmul.
"""
from .parser import LAParseError, parse
from .evaluator import LAInstance

__all__ = ["parse", "LAParseError", "LAInstance"]
