edits = []
