# Models package (drop-in for the reference's src/models).
