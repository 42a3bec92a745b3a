"""Parallelism: tensor parallel (xGMI one-shot all-reduce, leader/worker engine) -- tp.py."""
