"""provider.yaml loading and validation (REF ``src/config.ts:5-51``).

Behaviour kept byte-compatible with the reference:

* the file is YAML, read whole (``src/config.ts:9-10``);
* the nine required fields and the exact error strings
  ``Missing required field in client configuration: <field>`` and
  ``The "public" field in client configuration must be a boolean``
  (``src/config.ts:20-44``);
* no defaults, no coercion, unknown fields are kept and forwarded
  (``getAll``, ``src/config.ts:15-17``).

NEW: ``apiProvider: native`` selects the in-process MI355X
engine; optional engine fields (``tensorParallelSize``, ``maxBatchTokens``,
``kvCacheFraction``, ``weights``, ``seed``, ``maxTokens``, ...) are read by
:class:`symmetry_amd.engine.llm_engine.EngineConfig`; ``bootstrap`` lists
discovery nodes; ``SYMMETRY_*`` environment variables override fields for
bench harnesses.
"""
from __future__ import annotations

import os
from typing import Any

import yaml

REQUIRED_FIELDS = (
    "apiHostname",
    "apiPath",
    "apiPort",
    "apiProtocol",
    "apiProvider",
    "modelName",
    "path",
    "public",
    "serverKey",
)

DEFAULT_CONFIG_PATH = os.path.join(os.path.expanduser("~"), ".config", "symmetry", "provider.yaml")
ENV_PREFIX = "SYMMETRY_"
# optional fields (REF schema + native engine / provider options) an env override may name in any case
OPTIONAL_FIELDS = ("apiKey", "dataCollectionEnabled", "maxConnections", "name", "weights", "tokenizer",
                   "tensorParallelSize", "expertParallelSize", "maxBatchTokens", "maxModelLen", "kvCacheFraction",
                   "blockSize", "maxTokens", "seed", "device", "useGraphs", "numKvBlocks", "maxBacklog",
                   "decodeWeights", "prefillChunk", "strictServerAuth", "shareApiKey", "completionParser",
                   "metricsInterval", "metricsFile", "bootstrap", "listenHost", "listenPort", "serveHttp", "replicas")


class ConfigError(Exception):
    pass


class ConfigManager:
    def __init__(self, config_path: str, env: dict | None = None):
        with open(config_path, "r", encoding="utf-8") as f:
            config = yaml.safe_load(f)
        if not isinstance(config, dict):
            # js-yaml returns a scalar/undefined for such files; `field in config` then throws.
            raise ConfigError("Missing required field in client configuration: apiHostname")
        self.path = config_path
        self.config: dict[str, Any] = config
        self._apply_env(os.environ if env is None else env)
        self.validate()

    def _apply_env(self, env) -> None:
        for k, v in env.items():
            if not k.startswith(ENV_PREFIX):
                continue
            field = k[len(ENV_PREFIX):]
            for existing in list(self.config) + list(REQUIRED_FIELDS) + list(OPTIONAL_FIELDS):
                if existing.lower() == field.lower():
                    field = existing
                    break
            self.config[field] = yaml.safe_load(v) if v else v

    def validate(self) -> None:
        for field in REQUIRED_FIELDS:
            if field not in self.config:
                raise ConfigError(f"Missing required field in client configuration: {field}")
        if not isinstance(self.config["public"], bool):
            raise ConfigError('The "public" field in client configuration must be a boolean')

    def get(self, key: str, default: Any = None) -> Any:
        return self.config.get(key, default)

    def get_all(self) -> dict:
        return self.config

    getAll = get_all

    # convenience views ----------------------------------------------------------------------
    @property
    def is_native(self) -> bool:
        return str(self.config.get("apiProvider", "")).lower() == "native"


def default_config_text(name: str, config_dir: str, native: bool = False) -> str:
    """The provider.yaml written by the reference install script (``install.sh:35-50``)."""
    provider = "native" if native else "ollama"
    return (
        "# Symmetry Configuration\n"
        "apiHostname: localhost\n"
        "apiKey: \n"
        "apiPath: /v1/chat/completions\n"
        "apiPort: 11434\n"
        "apiProtocol: http\n"
        f"apiProvider: {provider}\n"
        "dataCollectionEnabled: true\n"
        "maxConnections: 10\n"
        "modelName: llama3.1:latest\n"
        f"name: {name}\n"
        f"path: {config_dir}\n"
        "public: true\n"
        "serverKey: 4b4a9cc325d134dee6679e9407420023531fd7e96c563f6c5d00fd5549b77435\n"
    )
