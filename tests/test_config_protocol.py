"""provider.yaml validation (REF src/config.ts) and the message / SSE codecs (REF src/utils.ts)."""
import json
import subprocess
import sys

import pytest

from symmetry_amd.config import REQUIRED_FIELDS, ConfigError, ConfigManager, default_config_text
from symmetry_amd.log import Logger, LogLevel
from symmetry_amd.protocol import codec, sse
from symmetry_amd.protocol.keys import API_PROVIDERS, SERVER_MESSAGE_KEYS, Keys

BASE = {
    "apiHostname": "localhost", "apiPath": "/v1/chat/completions", "apiPort": 11434, "apiProtocol": "http",
    "apiProvider": "ollama", "modelName": "llama3:8b", "path": "/tmp", "public": True,
    "serverKey": "4b4a9cc325d134dee6679e9407420023531fd7e96c563f6c5d00fd5549b77435",
}


def _write(tmp_path, cfg):
    import yaml

    p = tmp_path / "provider.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return str(p)


@pytest.mark.parametrize("missing", REQUIRED_FIELDS)
def test_each_required_field(tmp_path, missing):
    cfg = dict(BASE)
    del cfg[missing]
    with pytest.raises(ConfigError) as e:
        ConfigManager(_write(tmp_path, cfg), env={})
    assert str(e.value) == f"Missing required field in client configuration: {missing}"


def test_public_must_be_bool_and_unknown_fields_kept(tmp_path):
    cfg = dict(BASE, public="yes")
    with pytest.raises(ConfigError) as e:
        ConfigManager(_write(tmp_path, cfg), env={})
    assert str(e.value) == 'The "public" field in client configuration must be a boolean'
    cfg = dict(BASE, temperature=1, custom={"a": 1})
    cm = ConfigManager(_write(tmp_path, cfg), env={})
    assert cm.get_all()["temperature"] == 1 and cm.getAll()["custom"] == {"a": 1}
    assert cm.get("apiPort") == 11434  # no coercion
    assert cm.get("name") is None      # name is not required (REF quirk: all-zero seed)


def test_env_override(tmp_path):
    cm = ConfigManager(_write(tmp_path, dict(BASE)), env={"SYMMETRY_MODELNAME": "mixtral:8x7b",
                                                          "SYMMETRY_maxConnections": "3"})
    assert cm.get("modelName") == "mixtral:8x7b" and cm.get("maxConnections") == 3


def test_default_config_matches_install_script(tmp_path):
    import yaml

    d = yaml.safe_load(default_config_text("alice", "/home/alice/.config/symmetry"))
    assert d["maxConnections"] == 10 and d["dataCollectionEnabled"] is True and d["public"] is True
    assert d["modelName"] == "llama3.1:latest" and d["apiPort"] == 11434 and d["name"] == "alice"
    p = tmp_path / "provider.yaml"
    p.write_text(default_config_text("alice", str(tmp_path)))
    ConfigManager(str(p), env={})


def test_keys_and_providers():
    assert len(SERVER_MESSAGE_KEYS) == 16 and "conectionSize" in SERVER_MESSAGE_KEYS
    assert set(API_PROVIDERS.values()) == {"litellm", "llamacpp", "lmstudio", "ollama", "oobabooga", "openwebui"}


def test_create_message_js_semantics():
    assert codec.create_message(Keys.PONG) == '{"key":"pong"}'
    assert codec.create_message(Keys.INFERENCE_ENDED, "inference") == '{"key":"inferenceEnded","data":"inference"}'
    assert codec.create_message("x", None) == '{"key":"x","data":null}'
    b = codec.buffer_json(b"\x00\x01\xff")
    assert b == {"type": "Buffer", "data": [0, 1, 255]}
    assert codec.from_buffer_json(b) == b"\x00\x01\xff"
    assert codec.emitter_header("inference") == '{"symmetryEmitterKey":"inference"}'
    assert codec.safe_parse_json(b"{bad") is None
    assert codec.safe_parse_json('{"a":1}') == {"a": 1}


def _evt(content):
    return "data: " + json.dumps({"choices": [{"delta": {"content": content}}]}) + "\n\n"


def test_ref_stream_parsing_quirks():
    one = _evt("hi")
    assert sse.safe_parse_stream_response(one)["choices"][0]["delta"]["content"] == "hi"
    # two events in one chunk: the reference parses only the text between the first two "data:"
    # markers, so the first event is kept and the rest of the chunk is dropped from the completion
    assert sse.safe_parse_stream_response(one + _evt("there"))["choices"][0]["delta"]["content"] == "hi"
    assert sse.safe_parse_stream_response("not json") is None
    for prov in ("ollama", "openwebui", "litellm", "lmstudio", "oobabooga", "whatever"):
        assert sse.get_chat_data_from_provider(prov, sse.safe_parse_stream_response(one)) == "hi"
        assert sse.get_chat_data_from_provider(prov, None) == ""
    assert sse.get_chat_data_from_provider("llamacpp", {"content": "x"}) == "x"
    assert sse.get_chat_data_from_provider("llamacpp", {}) is None
    assert sse.get_chat_data_from_provider("litellm", {"choices": [{"delta": {"content": "undefined"}}]}) == ""


def test_sse_parser_and_encoder():
    p = sse.SSEParser()
    stream = _evt("a") + _evt("b") + "data: [DONE]\n\n"
    out = []
    for i in range(0, len(stream), 7):  # arbitrary chunk boundaries
        out += p.feed(stream[i:i + 7].encode())
    assert [sse.delta_of(e) for e in out] == ["a", "b", None]
    ev = sse.chunk_event("id1", "llama3:8b", "tok", role="assistant", created=1)
    obj = json.loads(ev[len("data: "):])
    assert obj["object"] == "chat.completion.chunk" and obj["choices"][0]["delta"] == {"role": "assistant",
                                                                                       "content": "tok"}
    assert sse.done_event() == "data: [DONE]\n\n"
    assert "error" in json.loads(sse.error_event("boom")[6:])


def test_logger_gating(capsys):
    lg = Logger()
    lg.set_log_level(LogLevel.WARNING)
    lg.info("hidden")
    lg.warning("shown")
    lg.debug("shown too")  # REF: debug is never gated
    out = capsys.readouterr().out
    assert "hidden" not in out and "shown" in out and "shown too" in out


def test_cli_version_and_init(tmp_path):
    r = subprocess.run([sys.executable, "-m", "symmetry_amd.cli", "--version"], capture_output=True, text=True)
    assert r.stdout.strip() == "1.0.0"
    p = tmp_path / "cfg" / "provider.yaml"
    r = subprocess.run([sys.executable, "-m", "symmetry_amd.cli", "--init", "-c", str(p)], capture_output=True,
                       text=True)
    assert r.returncode == 0 and p.exists()
    r = subprocess.run([sys.executable, "-m", "symmetry_amd.cli", "-c", str(tmp_path / "nope.yaml")],
                       capture_output=True, text=True)
    assert r.returncode == 1
