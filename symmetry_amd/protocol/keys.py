"""Protocol vocabulary (REF ``src/constants.ts``).

The 16 server message keys are reproduced verbatim, including the
misspelled ``conectionSize`` (``src/constants.ts:5``), because peers match on
the literal strings.  ``apiProviders`` gains ``native``: the
in-process MI355X engine; every other value keeps proxy mode.
"""
from __future__ import annotations

SERVER_MESSAGE_KEYS = {
    "challenge": "challenge",
    "conectionSize": "conectionSize",
    "heartbeat": "heartbeat",
    "inference": "inference",
    "inferenceEnded": "inferenceEnded",
    "join": "join",
    "joinAck": "joinAck",
    "leave": "leave",
    "newConversation": "newConversation",
    "ping": "ping",
    "pong": "pong",
    "providerDetails": "providerDetails",
    "reportCompletion": "reportCompletion",
    "requestProvider": "requestProvider",
    "sessionValid": "sessionValid",
    "verifySession": "verifySession",
}


class Keys:
    CHALLENGE = "challenge"
    CONECTION_SIZE = "conectionSize"
    HEARTBEAT = "heartbeat"
    INFERENCE = "inference"
    INFERENCE_ENDED = "inferenceEnded"
    JOIN = "join"
    JOIN_ACK = "joinAck"
    LEAVE = "leave"
    NEW_CONVERSATION = "newConversation"
    PING = "ping"
    PONG = "pong"
    PROVIDER_DETAILS = "providerDetails"
    REPORT_COMPLETION = "reportCompletion"
    REQUEST_PROVIDER = "requestProvider"
    SESSION_VALID = "sessionValid"
    VERIFY_SESSION = "verifySession"


API_PROVIDERS = {
    "LiteLLM": "litellm",
    "LlamaCpp": "llamacpp",
    "LMStudio": "lmstudio",
    "Ollama": "ollama",
    "Oobabooga": "oobabooga",
    "OpenWebUI": "openwebui",
}
NATIVE_PROVIDER = "native"

assert len(SERVER_MESSAGE_KEYS) == 16
