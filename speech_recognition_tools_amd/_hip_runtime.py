"""Which HIP runtime libfdlp_hip.so binds to when speech_recognition_tools_amd._lib first loads it.

TORCH (default): torch is imported first, so the library's libamdhip64.so.7 dependency resolves to the
copy torch-ROCm already loaded and torch tensors / streams and the kernels share ONE HIP runtime.  The
native JOB runner of compute-fdlp-feats uses no torch object: its CLI sets TORCH = False before anything
loads the library, so a cold JOB process does not spend ~2 s importing torch (the library then binds
the system ROCm runtime).  A torch-based API (FdlpPlan) refuses to run in such a process.
"""
TORCH = True
