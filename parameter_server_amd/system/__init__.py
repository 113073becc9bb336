"""Control-plane runtime: messages, transport, postoffice, executor, customers."""
