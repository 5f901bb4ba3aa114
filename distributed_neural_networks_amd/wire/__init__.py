"""Wire schema (reference ``node_service.proto``) and tensor codec."""
