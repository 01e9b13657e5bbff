# symmetry-amd installer for Windows (behaviour of the reference install.ps1:1-57).
# The native engine needs Linux + ROCm (MI355X); on Windows this installs PROXY mode: the provider
# relays requests to a local Ollama / OpenAI-compatible server exactly like the reference.
# Requires Python 3.10+, torch (CPU), and a C++ compiler + OpenSSL for the P2P transport module.
$ErrorActionPreference = "Stop"
$here = Split-Path -Parent $MyInvocation.MyCommand.Path

if (-not (Get-Command python -ErrorAction SilentlyContinue)) {
    Write-Host "Python is not installed. Please install Python 3.10+ and try again." -ForegroundColor Red
    exit 1
}
python -c "import torch" 2>$null
if ($LASTEXITCODE -ne 0) {
    Write-Host "PyTorch is not importable. Install torch first." -ForegroundColor Red
    exit 1
}

Write-Host "Building the P2P transport module..." -ForegroundColor Cyan
Push-Location $here
python -m symmetry_amd._build net
if ($LASTEXITCODE -ne 0) { Write-Host "native transport build failed" -ForegroundColor Red; Pop-Location; exit 1 }

Write-Host "Installing symmetry-cli..." -ForegroundColor Cyan
python -m pip install --user --no-deps --no-build-isolation -e .
if ($LASTEXITCODE -ne 0) { Write-Host "pip install failed" -ForegroundColor Red; Pop-Location; exit 1 }
Pop-Location

$configDir = Join-Path $env:USERPROFILE ".config\symmetry"
$configFile = Join-Path $configDir "provider.yaml"
python -m symmetry_amd.cli --init -c $configFile

Write-Host "Symmetry CLI installed successfully!" -ForegroundColor Green
Write-Host "Run 'symmetry-cli' to start the provider." -ForegroundColor Yellow
