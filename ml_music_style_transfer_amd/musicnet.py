"""Solo-piano selection over the MusicNet label files.

Drop-in for preprocessing/extract_piano_pieces_from_musicnet_dataset.py:10-24 (`main` keeps
its three arguments and its output file). The rule: a piece is solo piano when every note row
of its label CSV names instrument 1 and there is at least one row. The chosen CSV basenames go
one per line, in glob order, to `<output_file_basename>_<data_type>.txt`. Host-side file work
only (the csv module streams the one column; no device work, no pandas).
"""
import csv
import glob
import os

PIANO = 1.0  # MusicNet's instrument code for acoustic piano


def instrument_codes(label_csv):
    """The set of instrument codes in one MusicNet label file (its `instrument` column)."""
    with open(label_csv, newline="") as fh:
        return {float(row["instrument"]) for row in csv.DictReader(fh)}


def is_solo_piano(label_csv):
    return instrument_codes(label_csv) == {PIANO}


def main(path_to_musicnet, data_type, output_file_basename):
    """Write and return the basenames of the solo-piano label files of one split."""
    pattern = os.path.join(path_to_musicnet, data_type + "_labels", "*.csv")
    chosen = [os.path.basename(f) for f in glob.glob(pattern) if is_solo_piano(f)]
    with open(f"{output_file_basename}_{data_type}.txt", "w") as out:
        out.writelines(name + "\n" for name in chosen)
    return chosen


if __name__ == "__main__":
    import argparse
    cli = argparse.ArgumentParser(description="list the solo-piano pieces of a MusicNet split")
    cli.add_argument("--path-to-musicnet", default="../data/musicnet/")
    cli.add_argument("--data-type", default="test", choices=["train", "test"])
    cli.add_argument("--output-file-basename", default="piano_pieces")
    a = cli.parse_args()
    main(a.path_to_musicnet, a.data_type, a.output_file_basename)
