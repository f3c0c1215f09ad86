"""Socket front end (reference: src/pdbServer (PDBServer, ServerWork), src/mainServer (MasterMain,
WorkerMain, PDBMainServerInstance), src/communication (PDBCommunicator, SimpleRequest,
SimpleSendDataRequest), src/serverFunctionalities (CatalogServer, DispatcherServer,
QuerySchedulerServer, ...), scripts/startPseudoCluster.py / startMaster.sh / startWorkers.sh).

Deployment: ``torchrun --nproc-per-node N -m netsdb_amd.server.main --port 8108`` starts one process
per GPU.  Rank 0 (the "master") accepts client connections; every request is broadcast to all
ranks, which execute it SPMD on their PDBClient (catalog/storage/engine), and rank 0 answers.
Remote clients use :class:`RemotePDBClient` (same method names as PDBClient).  UDF libraries are
"registered" by module name (the analogue of registerType(libFoo.so)) and jobs are module
functions ``fn(client, **kwargs)`` that build and execute computations server-side.

Wire format: 4-byte big-endian length + UTF-8 JSON; tensors travel as {"__tensor__": [dtype,
shape, base64]}.  No pickle anywhere.
"""
from .protocol import recv_msg, send_msg
from .frontend import PDBFrontend, RemoteComp, RemotePDBClient, UDFRegistry, serve_worker

__all__ = ["PDBFrontend", "RemotePDBClient", "RemoteComp", "UDFRegistry", "serve_worker", "send_msg", "recv_msg"]
