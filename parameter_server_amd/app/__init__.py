"""Applications: linear methods (async SGD, Darlin, evaluation), hello world, main."""
