"""MusicNet solo-piano filter (preprocessing/extract_piano_pieces_from_musicnet_dataset.py:10-24).

A label file `<musicnet>/<data_type>_labels/<id>.csv` is a solo-piano piece when its
`instrument` column holds exactly one distinct value, 1 (piano). The names of those CSV files
are written one per line to `<output_file_basename>_<data_type>.txt`, in glob order like the
reference. Host-side file filtering (pandas CSV reads), no device work.
"""
import glob
import os

import pandas as pd

PIANO_INSTRUMENT_LABEL = 1


def main(path_to_musicnet, data_type, output_file_basename):
    path = os.path.join(path_to_musicnet, f"{data_type}_labels")
    label_files = glob.glob(f"{path}/*.csv")
    wav_file_list = []
    for file in label_files:
        instruments = list(set(pd.read_csv(file)['instrument'].values))
        if len(instruments) == 1 and instruments[0] == PIANO_INSTRUMENT_LABEL:
            wav_file_list.append(file)
    out = output_file_basename + f"_{data_type}.txt"
    with open(out, 'w') as f:
        for item in wav_file_list:
            f.write(f"{os.path.basename(item)}\n")
    return [os.path.basename(p) for p in wav_file_list]


if __name__ == '__main__':
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--path-to-musicnet", default='../data/musicnet/')
    ap.add_argument("--data-type", default='test', choices=['train', 'test'])
    ap.add_argument("--output-file-basename", default='piano_pieces')
    a = ap.parse_args()
    main(a.path_to_musicnet, a.data_type, a.output_file_basename)
