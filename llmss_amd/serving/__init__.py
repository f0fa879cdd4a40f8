"""Serving: pub/sub broker path (HTTP/gRPC producer -> broker -> TP consumer) and a direct gRPC
server on the tensor-parallel leader."""
