#!/usr/bin/env bash
# symmetry-amd installer (behaviour of the reference install.sh:1-59, MI355X-native build):
#   1. checks for python3 + torch (PyTorch-ROCm for the native engine; CPU torch suffices for proxy mode),
#   2. compiles the native code in-tree (gfx950 HIP kernels with hipcc, the C++ P2P transport with g++),
#   3. installs the package (console scripts symmetry-cli / symmetry-dht / symmetry-server / symmetry-client)
#      without touching the network (--no-deps --no-build-isolation),
#   4. writes ~/.config/symmetry/provider.yaml with the reference defaults if it does not exist.
# Usage: ./install.sh [--native]     (--native: apiProvider native = run the model on the local GPUs)
set -euo pipefail

here="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
native=""
[[ "${1:-}" == "--native" ]] && native="--native"

if ! command -v python3 >/dev/null 2>&1; then
  echo "python3 is not installed. Please install Python 3.10+ and try again." >&2
  exit 1
fi
if ! python3 -c "import torch" >/dev/null 2>&1; then
  echo "PyTorch is not importable. Install PyTorch-ROCm (GPU) or CPU torch (proxy mode) first." >&2
  exit 1
fi

echo "Building native extensions..."
( cd "$here" && python3 -m symmetry_amd._build net )
if command -v hipcc >/dev/null 2>&1 || [[ -x /opt/rocm/bin/hipcc ]]; then
  ( cd "$here" && PATH="/opt/rocm/bin:$PATH" python3 -m symmetry_amd._build kernels )
else
  echo "hipcc not found: GPU kernels skipped (proxy mode only)."
fi

echo "Installing symmetry-cli..."
python3 -m pip install --user --no-deps --no-build-isolation -e "$here" >/dev/null \
  || { echo "pip install failed" >&2; exit 1; }

config_dir="$HOME/.config/symmetry"
config_file="$config_dir/provider.yaml"
python3 -m symmetry_amd.cli --init $native -c "$config_file"

echo "Symmetry CLI installed successfully!"
echo "Run 'symmetry-cli' (or 'python3 -m symmetry_amd.cli') to start the provider."
