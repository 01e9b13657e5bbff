"""Native runtime pieces around the GPU path (csrc/runtime, built into ``_runtime.so``)."""
