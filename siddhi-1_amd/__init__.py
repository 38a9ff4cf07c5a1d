"""siddhi-1_amd — MI355X-native engine for Siddhi's partitioned pattern / sequence queries.

Host side of the drop-in seam described in include/siddhi_gpu.h: a SiddhiQL-subset compiler that
lowers a pattern/sequence query to the engine IR (include/siddhi_gpu_ir.h), a mirror of the
reference's public API (SiddhiManager / SiddhiAppRuntime / InputHandler / callbacks), and the
ctypes binding of the HIP engine library (lib/libsiddhi_gpu.so, built from csrc/).

The directory name is not a Python identifier; import it with
``importlib.import_module("siddhi-1_amd")``.
"""
from .runtime import (Event, InputHandler, QueryCallback, ColumnarQueryCallback, SiddhiAppRuntime,  # noqa: F401
                      SiddhiManager,
                      StreamCallback, StringDictionary, InMemoryPersistenceStore,
                      CannotRestoreSiddhiAppStateException, NoPersistenceStoreException)
from .compiler import compile_query, SiddhiAppCreationException  # noqa: F401
from .siddhiql import parse_app, SiddhiParserException  # noqa: F401
from .native import NativeEngine, EngineError, load_hip_library, load_library, jit_check, HIP_LIBRARY  # noqa: F401
